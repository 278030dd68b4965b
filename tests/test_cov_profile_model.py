"""The stated collective cost model of the rank projection (tools/cov_profile.py: collective_model):
an all-to-all of the 32-B rows that leave their rank (measured per rank: the records a rank keeps for
its own cells never cross xGMI) plus an all-gather of the owners' f64
x columns, over a stated xGMI rate, with a fixed latency per collective (three of them)."""
import importlib.util
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _model():
    spec = importlib.util.spec_from_file_location("cov_profile", os.path.join(REPO, "tools", "cov_profile.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.collective_model


class _Grid:
    nx, ny, nz = 256, 256, 1


def test_collective_model_arithmetic(monkeypatch):
    monkeypatch.setenv("XGMI_GBS", "300")
    monkeypatch.setenv("COLL_US", "25")
    m = _model()([200_000, 180_000], [150_000, 210_000], _Grid(), 8)
    a2a = 210_000 * 32  # the largest remote sender or receiver
    ag = (256 + 7) // 8 * 256 * 8 * 7  # the other owners' columns, f64
    assert m["a2a_bytes_max"] == int(a2a)
    assert m["allgather_bytes_in"] == ag
    assert abs(m["ms_all_to_all"] - round(0.05 + a2a / 300e9 * 1e3, 4)) < 1e-9
    assert abs(m["ms_all_gather"] - round(0.025 + ag / 300e9 * 1e3, 4)) < 1e-9
    assert abs(m["ms_total"] - round(m["ms_all_to_all"] + m["ms_all_gather"], 4)) < 1e-3


def test_collective_model_one_rank_moves_nothing():
    m = _model()([0], [0], _Grid(), 1)
    assert m["a2a_bytes_max"] == 0 and m["allgather_bytes_in"] == 0
