set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_files.py tests/test_gpu_shim.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_files.log 2>&1 &&
timeout -k 10 200 python tools/files_bench.py --batch 30 --batches 6 > gpurun_out/files_bench.json 2> gpurun_out/files_bench.err &&
(export TMPDIR=/tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_files -o kt --output-format csv -- python3 tools/files_bench.py --batch 30 --batches 6 > gpurun_out/files_bench_prof.json 2>&1)
rc=$?
tail -5 gpurun_out/pytest_files.log; cat gpurun_out/files_bench.json
exit $rc
