"""The closed-form signal power used on the device (coverage.hip power_sparse), restated here in
Python and checked against the reference computation (np.convolve 'same' + np.nonzero,
coverage.py:45-52 / main.py:46-55) on sparse impulse responses.  CPU only."""
import math

import numpy as np
import pytest

from oracle import oracle as orc
from rf_ray_tracing_warp_amd.coverage import phase_step


def power_closed_form(bins, amps, n, window):
    """Python twin of power_sparse(): bins ascending and unique."""
    if len(bins) == 0:
        return float("nan")
    half = (n - 1) // 2
    al = phase_step(window, n)
    s = [max(0, m - half) for m in bins]
    e = [min(n - 1, m + (n - 1 - half)) for m in bins]
    total, count = 0.0, 0
    i_s = i_e = 0
    x = 0
    K = len(bins)
    while True:
        nstart = 0
        while i_s < K and s[i_s] <= x:
            i_s += 1
            nstart += 1
        while i_e < i_s and e[i_e] < x:
            i_e += 1
        alone = i_s - i_e == 1 and nstart == 1 and bins[i_s - 1] - half == x
        nx = n
        if i_s < K:
            nx = min(nx, s[i_s])
        if i_e < i_s:
            nx = min(nx, e[i_e] + 1)
        if i_e < i_s:
            P = sum(amps[k] * math.cos(al * (half - bins[k])) for k in range(i_e, i_s))
            Q = sum(amps[k] * math.sin(al * (half - bins[k])) for k in range(i_e, i_s))
            u, v = x, nx - 1
            L = v - u + 1
            D = math.sin(L * al) * math.cos((u + v) * al) / math.sin(al)
            E = math.sin(L * al) * math.sin((u + v) * al) / math.sin(al)
            total += P * P * 0.5 * (L - D) + Q * Q * 0.5 * (L + D) + 2 * P * Q * 0.5 * E
            count += L - (1 if alone else 0)
        if nx >= n:
            break
        x = nx
    return total / count if count else float("nan")


def _ir(bins, amps, n):
    ir = np.zeros(n)
    ir[bins] = amps
    return ir


@pytest.mark.parametrize("seed", range(12))
def test_closed_form_matches_numpy_convolve(seed):
    rng = np.random.default_rng(seed)
    n = [10000, 20000, 1001, 10][seed % 4]
    win = 100e-9 if n != 20000 else 200e-9
    K = int(rng.integers(1, 40))
    bins = np.sort(rng.choice(n, size=min(K, n), replace=False))
    amps = rng.uniform(1e-7, 1e-5, len(bins))
    ref = orc.signal_power(_ir(bins, amps, n), win)
    got = power_closed_form(bins.tolist(), amps.tolist(), n, win)
    assert abs(got - ref) <= 1e-9 * abs(ref), (got, ref)


@pytest.mark.parametrize("bins", [[6637], [4999], [5000], [0], [9999], [4999, 5000], [7000, 7001, 9999], [12, 9998]])
def test_closed_form_edges(bins):
    n, win = 10000, 100e-9
    amps = [1.25e-7 * (i + 1) for i in range(len(bins))]
    ref = orc.signal_power(_ir(np.array(bins), np.array(amps), n), win)
    got = power_closed_form(bins, amps, n, win)
    assert abs(got - ref) <= 1e-9 * abs(ref), (bins, got, ref)


def test_closed_form_empty_is_nan():
    assert math.isnan(power_closed_form([], [], 10000, 100e-9))
    assert math.isnan(orc.signal_power(np.zeros(10000), 100e-9))
