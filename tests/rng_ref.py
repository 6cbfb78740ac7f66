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
