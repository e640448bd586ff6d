mkdir -p gpurun_out/r04j
timeout -k 10 400 python -u -m pytest tests/test_gpu_band.py -x -v --timeout 200 --timeout-method thread -s > gpurun_out/r04j/band_all.log 2>&1; rc=$?
grep -E "windows [0-9]+, band|PASSED|FAILED|passed|failed|Error" gpurun_out/r04j/band_all.log | tail -30
exit $rc
