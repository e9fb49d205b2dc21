"""BlsGpuVerifier's pubkey queue on the CPU, against a mock addon (tests/node/flush_mock.js):
keys packed into contiguous runs by the hook and uploaded in index order, a device error keeps
the failed run and every later one queued, only an undecodable-key status drops its run, and the
flush itself holds the event loop well under a call's latency (VERDICT r04 next #4;
state-transition/src/cache/epochContext.ts:702-705, pubkeyCache.ts:56-77).  The mock stands in
for blsgpu.node only; the same logic runs against the real addon in tests/node/wiring.js."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ADDON = os.path.join(HERE, "..", "lodestar_amd", "node", "blsgpu.node")


@pytest.mark.skipif(shutil.which("node") is None, reason="no Node")
def test_pubkey_flush_against_mock_addon():
    if not os.path.exists(ADDON):  # the mock is installed under the addon's resolved path
        pytest.skip("blsgpu.node not built")
    out = subprocess.run(["node", "--expose-gc", os.path.join(HERE, "node", "flush_mock.js")], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "flush mock ok" in out.stdout
