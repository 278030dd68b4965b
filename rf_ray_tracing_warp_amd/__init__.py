"""rf_ray_tracing_warp_amd -- MI355X-native drop-in for the Warp hot path of rf_ray_tracing_warp.

Public surface (mirrors the reference):
    Tracer(mesh, light_speed_mps, sample_rate_hz, sample_window_s, max_bounces, tx_num_rays)
        .compute_cir(tx_pos, tx_power, rx_pos, rx_radius) -> (paths, impulse_response)
    load_mesh / load_stl / sphere            (trimesh stand-ins, mesh.py)
    to_dbm, signal_power                     (main.py / coverage.py helpers, power.py)
    coverage_map                              (coverage.py driver, coverage.py)
"""
from .mesh import TriMesh, icosphere, load_mesh, load_stl, sphere  # noqa: F401
from .power import signal_power, to_dbm  # noqa: F401
from .tracer import Tracer  # noqa: F401

__version__ = "0.1.0"
