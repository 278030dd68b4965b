"""The library's remaining A/B switches (read once per process; DESIGN.md "switch inventory"):
their non-default paths give the default paths' bits.  RFRT_K2_BOX=0 (every face at bounces >= 1
instead of the wave's bundle-box candidates), RFRT_K2_LPT=0 (chunks in order instead of the
cached longest-first schedule) and RFRT_TRAJ_SPLIT_MAX=0 (one lane per ray for a rank plan's BVH
trajectories instead of four) run in a child process started with them set (tests/_switch_child.py).
RFRT_COV_CLEAR and RFRT_COV_RXFIRST have their own equivalence tests (test_gpu_coverage.py,
test_gpu_poison.py)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_switch_paths_are_bit_identical(require_gpu):
    env = dict(os.environ, RFRT_K2_BOX="0", RFRT_K2_LPT="0", RFRT_TRAJ_SPLIT_MAX="0")
    r = subprocess.run([sys.executable, os.path.join(HERE, "_switch_child.py")], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "switch paths ok" in r.stdout
