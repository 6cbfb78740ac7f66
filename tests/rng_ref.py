"""numpy restatement of the device RNG (physics.hip: threefry2x32 / uniform01) for tests.

threefry2x32-20 is the Random123 generator jax.random uses; `uniform01` maps 32 random bits to
[0, 1) with jax.random.uniform's float32 mapping ((bits >> 9) | 0x3f800000) - 1."""
import numpy as np

_ROT = (13, 15, 26, 6, 17, 29, 16, 24)
M32 = 0xFFFFFFFF


def threefry2x32(k0, k1, x0, x1):
    k0, k1 = np.uint64(k0) & M32, np.uint64(k1) & M32
    x0 = np.asarray(x0, np.uint64) & M32
    x1 = np.asarray(x1, np.uint64) & M32
    ks = [k0, k1, (k0 ^ k1 ^ np.uint64(0x1BD11BDA)) & M32]
    x0 = (x0 + ks[0]) & M32
    x1 = (x1 + ks[1]) & M32
    for i in range(5):
        for j in range(4):
            r = np.uint64(_ROT[(i & 1) * 4 + j])
            x0 = (x0 + x1) & M32
            x1 = ((x1 << r) | (x1 >> (np.uint64(32) - r))) & M32
            x1 = x1 ^ x0
        x0 = (x0 + ks[(i + 1) % 3]) & M32
        x1 = (x1 + ks[(i + 2) % 3] + np.uint64(i + 1)) & M32
    return x0, x1


def uniform01(seed: int, counter: int, env, idx):
    k0, k1 = threefry2x32(seed & M32, (seed >> 32) & M32, counter & M32, (counter >> 32) & M32)
    b0, _ = threefry2x32(int(k0), int(k1), env, idx)
    bits = ((b0 >> np.uint64(9)) | np.uint64(0x3F800000)).astype(np.uint32)
    return bits.view(np.float32) - np.float32(1.0)


def reset_noise(seed: int, counter: int, nenv: int, ndraw: int) -> np.ndarray:
    env = np.repeat(np.arange(nenv, dtype=np.uint64), ndraw)
    idx = np.tile(np.arange(ndraw, dtype=np.uint64), nenv)
    return uniform01(seed, counter, env, idx).reshape(nenv, ndraw)


# ------------------------------------------------------------------ jax.random on threefry2x32
# Partitionable layout (jax >= 0.5 default): element i of a draw / split = threefry(key, (0, i)).
# Original layout: a draw of n words is threefry over (iota halves) of iota(n) padded with a 0.
PARTITIONABLE, ORIGINAL = 1, 2


def _words(key, n, mode):
    k0, k1 = int(key[0]), int(key[1])
    if mode == PARTITIONABLE:
        x0, x1 = threefry2x32(k0, k1, np.zeros(n, np.uint64), np.arange(n, dtype=np.uint64))
        return x0, x1
    c = np.arange(n, dtype=np.uint64)
    if n % 2:
        c = np.concatenate([c, np.zeros(1, np.uint64)])
    h = c.size // 2
    y0, y1 = threefry2x32(k0, k1, c[:h], c[h:])
    return np.concatenate([y0, y1])[:n], None


def jax_split(key, num, mode=PARTITIONABLE):
    """jax.random.split(key, num) -> uint32 [num, 2]."""
    if mode == PARTITIONABLE:
        x0, x1 = _words(key, num, mode)
        return np.stack([x0, x1], 1).astype(np.uint32)
    w, _ = _words(key, 2 * num, mode)
    return w.reshape(num, 2).astype(np.uint32)


def jax_uniform(key, n=None, mode=PARTITIONABLE):
    """jax.random.uniform(key, (n,)) (n=None: shape ()) as float32."""
    m = 1 if n is None else n
    if mode == PARTITIONABLE:
        x0, x1 = _words(key, m, mode)
        bits = x0 ^ x1
    else:
        bits, _ = _words(key, m, mode)
    f = (((bits >> np.uint64(9)) | np.uint64(0x3F800000)).astype(np.uint32)).view(np.float32) - np.float32(1.0)
    return f[0] if n is None else f


def jax_reset_noise(keys, nj, nv, mode=PARTITIONABLE):
    """single_reset's draws (src/envs.py:117-141) from per-env keys [B, 2], in the device layout
    [joint uniforms (nj) | velocity uniforms (nv) | flip uniform | initial-speed uniform]."""
    out = []
    for key in np.asarray(keys, np.uint32):
        k1, k2, k3, k4 = jax_split(key, 4, mode)
        out.append(np.concatenate([jax_uniform(k1, nj, mode), jax_uniform(k2, nv, mode),
                                   [jax_uniform(k3, None, mode), jax_uniform(k4, None, mode)]]))
    return np.array(out, np.float32)
