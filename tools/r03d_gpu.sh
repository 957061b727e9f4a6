set -o pipefail
mkdir -p gpurun_out/r03d
timeout -k 10 600 python -u -m pytest tests/test_system_dropin.py tests/test_multi_device.py tests/test_full_size.py tests/test_engine_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "system or c4 or System or multi or split or full" > gpurun_out/r03d/pytest.log 2>&1; echo "pytest rc $?"; tail -5 gpurun_out/r03d/pytest.log
PE_API_PROF=1 timeout -k 10 120 python -u tools/c4_probe.py > gpurun_out/r03d/c4_probe.txt 2>&1; echo "probe rc $?"; tail -30 gpurun_out/r03d/c4_probe.txt
bash tools/c4_pmc.sh
