"""The chain kernel's synchronisation under wave skew: the skew build
(mcmc-in-tonga_amd/libtdstar_skew.so, -DTD_CHAIN_SKEW) puts one wave to sleep for longer than a phase
after every block barrier and barrier-free phase end, rotating with the iteration; a shared word read
without a synchronisation that orders it then shows up as a state that differs from the host engine's,
or a spin wait that gives up.  The device chain must still follow the host engine bit for bit on every
shape of test_gpu_chain (TD_inversion_function.jl:70-274), the 8-cell model at max_cells 12 -- whose
births at the cap are inactive proposals -- included."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SKEW = os.path.join(ROOT, "mcmc-in-tonga_amd", "libtdstar_skew.so")


@pytest.mark.timeout(240)
def test_chain_follows_host_under_wave_skew():
    assert os.path.exists(SKEW), "the skew build is made by __graft_entry__.build() (make all)"
    env = dict(os.environ, TD_LIB_PATH=SKEW)
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "skew_worker.py")], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=220, cwd=ROOT)
    text = p.stdout.decode(errors="replace")
    rows = [json.loads(x) for x in text.splitlines() if x.startswith("{")]
    assert p.returncode == 0 and len(rows) == 16, text[-3000:]
    assert all(r["same"] and r["guard"] == 0 for r in rows), rows
