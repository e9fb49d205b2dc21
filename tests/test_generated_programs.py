"""The generated point / Miller programs in lodestar_amd/csrc match their generators
(tools/gen_tmiller.py, gen_tcurve.py, gen_tg1.py): each generator runs in a scratch copy of the
tree layout and its output must equal the committed header byte for byte, so a formula edit
cannot ship without its regenerated table (the generators' own asserts check every
instruction's bounds and the no-read-and-write-in-one-round rule while they run)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [("gen_tmiller.py", "bgv_tmiller_prog.h"), ("gen_tcurve.py", "bgv_tcurve_prog.h"),
         ("gen_tg1.py", "bgv_tg1_prog.h")]


@pytest.mark.parametrize("gen,header", CASES)
def test_generated_header_is_current(tmp_path, gen, header):
    tools = tmp_path / "tools"
    tools.mkdir()
    (tmp_path / "lodestar_amd" / "csrc").mkdir(parents=True)
    for f in ("gen_tmiller.py", gen):
        shutil.copy(os.path.join(ROOT, "tools", f), tools / f)
    subprocess.run([sys.executable, str(tools / gen)], check=True, capture_output=True, timeout=300)
    got = (tmp_path / "lodestar_amd" / "csrc" / header).read_text()
    want = open(os.path.join(ROOT, "lodestar_amd", "csrc", header)).read()
    assert got == want, "%s is stale: run python tools/%s" % (header, gen)
