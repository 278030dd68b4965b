"""Received signal power helpers of the reference scripts (host, NumPy).

``signal_power`` restates main.py:39-52 / coverage.py:45-52: convolve the impulse response
with a sampled 2.4 GHz sine ('same' mode), keep the exactly-nonzero samples (the ``[:10000]``
slice acts on the tuple returned by np.nonzero and is a no-op), mean of squares.
``to_dbm`` is main.py:12-13.  The coverage path computes the same quantity on the device in
closed form (coverage.hip); this host version is the reference semantics for single CIRs.
"""
from __future__ import annotations

import numpy as np

CARRIER_HZ = 2.4e9  # main.py:45, coverage.py:46


def to_dbm(power):
    with np.errstate(divide="ignore", invalid="ignore"):
        return 10 * np.log10(power / 1e-3)


def signal_power(impulse_response, sample_window_s):
    ir = np.asarray(impulse_response, dtype=np.float64)
    with np.errstate(all="ignore"):
        time = np.linspace(0, sample_window_s, ir.shape[0])
        signal_tx = np.sin(2 * np.pi * CARRIER_HZ * time)
        signal_rx = np.convolve(ir, signal_tx, mode="same")
        r = np.nonzero(signal_rx)
        signal_rx = signal_rx[r]
        return np.sum(signal_rx ** 2) / signal_rx.shape[0]
