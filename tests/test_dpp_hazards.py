"""CPU: the build-time DPP hazard checker (tools/dpp_hazards.py) flags a DPP read one wait state
after the VALU write of its source and passes two."""
import os
import subprocess
import sys

from tests.conftest import ROOT

TOOL = os.path.join(ROOT, "tools", "dpp_hazards.py")

HEAD = "0000000000001000 <_ZN3svh12_GLOBAL__N_119pipe_viterbi_kernelILi2ELi4ELb0ELi0EEEv>:\n"


def run(tmp_path, body):
    p = tmp_path / "k.s"
    p.write_text(HEAD + body)
    return subprocess.run([sys.executable, TOOL, str(p)], capture_output=True, text=True)


def test_one_wait_state_is_a_hazard(tmp_path):
    r = run(tmp_path, "\tv_add_f32_e32 v139, v1, v2\n"
                      "\tv_add_f32_e32 v160, v3, v4\n"
                      "\tv_add_f32_dpp v166, v139, v141 row_ror:9 row_mask:0xf bank_mask:0xf\n")
    assert r.returncode == 1 and "HAZARD" in r.stdout


def test_two_wait_states_pass(tmp_path):
    r = run(tmp_path, "\tv_add_f32_e32 v139, v1, v2\n"
                      "\tv_add_f32_e32 v160, v3, v4\n"
                      "\ts_nop 0\n"
                      "\tv_add_f32_dpp v166, v139, v141 row_ror:9 row_mask:0xf bank_mask:0xf\n")
    assert r.returncode == 0 and "hazards 0" in r.stdout


def test_built_kernel_was_checked():
    """The tree's build of pipe.hip passed the check (make writes build/pipe.hazards)."""
    f = os.path.join(ROOT, "build", "pipe.hazards")
    if os.path.exists(f):
        assert "hazards 0" in open(f).read()
