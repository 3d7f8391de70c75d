"""Run-to-run determinism of the network with other processes on the same GPU (r04: a grid-stride
version of i2pc_ln_apply gave different hidden states between identical forwards when a second
process shared the card, while each single-process run was deterministic).  Two processes each run
the Depth-Anything-V2-Small pipeline several times on their own images; every forward of a process
must be bit-identical to its first (tools/det_rep.py is the same check with more repetitions)."""
import os
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")
pytestmark = [pytest.mark.gpu, pytest.mark.two_process]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.xfail(strict=False, reason="open defect, DESIGN.md §2.2 'two-process nondeterminism': under "
                   "two processes per GPU the 256x128 LN-fold QKV part (DA-v2 columns 1024-1151) differs "
                   "run to run; single-process runs (the deployment configuration) are deterministic")
def test_two_processes_deterministic():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "det_rep.py"), "2", "10", "0"],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    lines = [l for l in r.stdout.splitlines() if l.startswith("proc")]
    assert r.returncode == 0 and len(lines) == 2, r.stdout[-2000:] + r.stderr[-2000:]
    for l in lines:
        assert ": 0 of 9 runs differ" in l and "hs differ [0, 0, 0, 0]" in l, l
