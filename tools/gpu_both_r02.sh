bash tools/gpu_chol_diag.sh && bash tools/gpu_c5_pipe.sh
