bash tools/gpu_c2_tall.sh && bash tools/gpu_prof_c5_r02.sh
