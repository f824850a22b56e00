cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_vjp.py -q -x --timeout 120 --timeout-method thread > gpurun_out/vjp.log 2>&1; rc=$?; tail -3 gpurun_out/vjp.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/wide_train_compare.py cfg4 > gpurun_out/wcmp.log 2>&1; rc=$?; tail -3 gpurun_out/wcmp.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_w -o run --output-format csv -- python tools/prof_target.py --workload cfg4 --mode train --launches 5 > gpurun_out/prof_w.log 2>&1; echo rc=$?
