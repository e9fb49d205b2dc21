"""The Node package entry (lodestar_amd/node/index.js): verifier selection of
chain/chain.ts:189-192 with the GPU branch (createBlsVerifier), the chain options and CLI
flags (chainOptions.js), on CPU with stand-in CPU verifiers; on the GPU the factory's GPU
branch verifies a signature set through the N-API addon with the pubkey hook installed."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SCRIPT = os.path.join(HERE, "node", "wiring.js")
NODE = shutil.which("node")


def _run(env_extra=None):
    env = dict(os.environ, **(env_extra or {}))
    return subprocess.run([NODE, SCRIPT], capture_output=True, text=True, timeout=180, env=env)


@pytest.mark.skipif(NODE is None, reason="node not installed")
def test_wiring_selection_and_options():
    r = _run()
    assert r.returncode == 0, r.stderr
    assert "wiring ok" in r.stdout


@pytest.mark.gpu
@pytest.mark.skipif(NODE is None, reason="node not installed")
def test_wiring_gpu_branch_verifies():
    from lodestar_amd import build
    if not os.path.exists(build.NODE_ADDON):
        pytest.fail("blsgpu.node not built")
    r = _run({"BGV_WIRING_GPU": "1"})
    assert r.returncode == 0, r.stderr + r.stdout
    assert "wiring ok" in r.stdout
