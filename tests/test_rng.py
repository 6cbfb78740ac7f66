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


def test_jax_split_known_answers():
    """jax.random.split(jax.random.PRNGKey(0)) as JAX prints it: [[1797259609 2579123966]
    [928981903 3453687069]] with jax_threefry_partitionable (default since jax 0.5; the reference
    pins 0.7.2), [[4146024105 967050713] [2718843009 1272950319]] in the original layout."""
    from rng_ref import ORIGINAL, PARTITIONABLE, jax_split
    np.testing.assert_array_equal(jax_split((0, 0), 2, PARTITIONABLE), [[1797259609, 2579123966], [928981903, 3453687069]])
    np.testing.assert_array_equal(jax_split((0, 0), 2, ORIGINAL), [[4146024105, 967050713], [2718843009, 1272950319]])


def test_jax_uniform_layouts():
    from rng_ref import ORIGINAL, PARTITIONABLE, jax_uniform
    for mode in (PARTITIONABLE, ORIGINAL):
        u = jax_uniform((7, 42), 4099, mode)
        assert u.dtype == np.float32 and 0.0 <= u.min() and u.max() < 1.0 and abs(u.mean() - 0.5) < 0.02
        # a shape-() draw is element 0 of any draw in the partitionable layout; in the original one it
        # is the first word of threefry over the padded pair (0, 0)
        s = jax_uniform((7, 42), None, mode)
        if mode == PARTITIONABLE:
            assert s == u[0]
