set -u
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_model_gpu.py -k "pool_squeeze" -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_r04d.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_r04d.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_layers.sh r04d f32 psold cur psold cur
grep -E "^\[|pool" gpurun_out/ab_r04d.txt
