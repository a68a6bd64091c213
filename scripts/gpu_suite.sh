set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/full_tests.log 2>&1 || { tail -60 gpurun_out/full_tests.log; exit 1; }
tail -3 gpurun_out/full_tests.log
