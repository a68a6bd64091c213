"""The C ABI from C++ (tests/capi/capi_check.cpp, built by __graft_entry__.build()): one PPO
step through trlx_ppo_experience_fused + trlx_ppo_loss_fused, with no Python or torch in the
process, against the program's own double-precision restatement of the reference arithmetic
(modeling.py:37-41, ppo_orchestrator.py:163-167, ppo_models.py:121-199)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "capi", "capi_check")


def test_capi_consumer_step_matches_host_restatement():
    if not os.path.exists(EXE):
        raise RuntimeError(f"{EXE} is not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "capi_check ok" in r.stdout
