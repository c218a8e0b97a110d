#!/bin/bash
# The C12 split (SCS_CHOL_C12_SPLIT): the Cholesky bit-identity / backward-error tests, then the factor
# probe with the split off / on (and the m = 16384 bulk skip set on top), one process each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/r04/c12}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "cholesky or lookahead or bounded or diag_pipe or default_path or solve" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  SCS_CHOL_C12_SPLIT=$v timeout -k 10 120 ./tools/probes/bin/probe_chol_c12 > $O/probe_split$v.log 2>&1 || exit 1
  echo "split=$v"; grep "factor\|solve" $O/probe_split$v.log
done
SCS_CHOL_BULK_SKIP=0x20 timeout -k 10 120 ./tools/probes/bin/probe_chol_c12 > $O/probe_split1_skip.log 2>&1 || exit 1
echo "split=1 skip=0x20"; grep "factor" $O/probe_split1_skip.log
