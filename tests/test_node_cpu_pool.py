"""The Node gossip bench's CPU row (a same-shape CPU figure): the C++
restatement of the verify path behind CpuPoolVerifier (BlsMultiThreadWorkerPool's buffering,
chain/bls/multithread/index.ts:255-412) gives the committed goldens' verdicts through N-API.
Test infrastructure only; the GPU rows of tests/node/gossip_bench.js run on the GPU box."""
import json
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("node") is None or not os.path.exists("/usr/include/node/node_api.h"),
                    reason="no Node / N-API headers")
def test_cpu_pool_verifier_goldens():
    import sys
    sys.path.insert(0, os.path.join(HERE, "node"))
    subprocess.check_call([sys.executable, os.path.join(HERE, "node", "build_cpu.py")], stdout=subprocess.DEVNULL)
    out = subprocess.run(["node", os.path.join(HERE, "node", "cpu_pool_check.js")], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["ok"] and r["checked"] >= 20
