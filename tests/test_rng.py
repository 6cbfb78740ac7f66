"""Device RNG restatement pinned by the Random123 threefry2x32-20 known-answer vectors."""
import numpy as np

from rng_ref import reset_noise, threefry2x32


def test_threefry_kat():
    # Random123 kat_vectors: threefry2x32_20
    assert tuple(int(v) for v in threefry2x32(0, 0, 0, 0)) == (0x6B200159, 0x99BA4EFE)
    assert tuple(int(v) for v in threefry2x32(0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF)) == (0x1CB996FC, 0xBB002BE7)
    assert tuple(int(v) for v in threefry2x32(0x13198A2E, 0x03707344, 0x243F6A88, 0x85A308D3)) == (0xC4923A9C, 0x483DF7A0)


def test_uniform_range_and_moments():
    u = reset_noise(42, 7, 4096, 50)
    assert u.dtype == np.float32 and u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 3e-3 and abs(u.var() - 1 / 12) < 2e-3
    # different counters / envs give different streams
    assert not np.array_equal(reset_noise(42, 8, 4, 50), reset_noise(42, 7, 4, 50))
    assert not np.array_equal(u[0], u[1])
