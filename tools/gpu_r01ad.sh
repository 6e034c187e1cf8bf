set -e
R=$GRAFT_REPO_ROOT; RUN=${RUN:-r01ad}; O=$R/gpurun_out/$RUN; mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/misaligned_ar.py > $O/misaligned_ar.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_collectives.py -x -q --timeout 300 --timeout-method thread > $O/pytest_coll.log 2>&1
