set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/full_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/full_pytest.log; exit $rc
