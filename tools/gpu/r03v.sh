set -o pipefail
O=gpurun_out/r03v; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_r03.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { echo failed; tail -30 $O/pytest.txt; exit 1; }
tail -5 $O/pytest.txt
