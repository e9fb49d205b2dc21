set -o pipefail
mkdir -p gpurun_out/r03a
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r03a/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r03a/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc stop"; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03a/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/r03a/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err || { echo bench failed; tail gpurun_out/r03a/bench.err; exit 1; }
cat gpurun_out/r03a/bench.json
echo pytest_rc=$rc
