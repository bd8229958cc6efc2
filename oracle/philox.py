"""numpy Philox4x32-10 and the HIP normal transform — TEST INFRASTRUCTURE ONLY.

Restates ``samplers_amd/csrc/sp_common.h`` (philox4x32_10, u01, philox_normal4)
so the in-kernel noise stream can be checked: the 32-bit Philox words
bit-exactly (plus the Random123 known-answer vectors), the normals to a few
ulp (device v_log_f32 / v_sin_f32 / v_cos_f32 vs fp64 here).
"""

from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr: np.ndarray, key: tuple[int, int]) -> np.ndarray:
    """ctr: (..., 4) uint32; returns (..., 4) uint32."""
    c = np.asarray(ctr, dtype=np.uint32).copy()
    k0 = np.uint32(key[0])
    k1 = np.uint32(key[1])
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = M0 * c[..., 0].astype(np.uint64)
            p1 = M1 * c[..., 2].astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & MASK32).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & MASK32).astype(np.uint32)
            c = np.stack([hi1 ^ c[..., 1] ^ k0, lo1, hi0 ^ c[..., 3] ^ k1, lo0], axis=-1)
            k0 = np.uint32(k0 + W0)
            k1 = np.uint32(k1 + W1)
    return c


def u01(u: np.ndarray) -> np.ndarray:
    return ((u >> np.uint32(9)).astype(np.float32) + np.float32(0.5)) * np.float32(2.0**-23)


def normals(seed: int, step: int, sample: int, n: int) -> np.ndarray:
    """The n standard normals the HIP kernels draw for (seed, step, sample)."""
    groups = (n + 3) // 4
    s = np.uint64(step & 0xFFFFFFFFFFFFFFFF)
    ctr = np.zeros((groups, 4), dtype=np.uint32)
    ctr[:, 0] = np.arange(groups, dtype=np.uint64).astype(np.uint32)
    ctr[:, 1] = np.uint32(sample & 0xFFFFFFFF)
    ctr[:, 2] = np.uint32(int(s) & 0xFFFFFFFF)
    ctr[:, 3] = np.uint32(int(s) >> 32)
    r = philox4x32_10(ctr, (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF))
    u = u01(r).astype(np.float64)
    rad0 = np.sqrt(-2.0 * np.log(u[:, 0]))
    rad1 = np.sqrt(-2.0 * np.log(u[:, 2]))
    # the device takes sin/cos of 2*pi*u exactly in revolutions (v_sin_f32 / v_cos_f32)
    th0 = 2.0 * np.pi * u01(r[:, 1]).astype(np.float64)
    th1 = 2.0 * np.pi * u01(r[:, 3]).astype(np.float64)
    z = np.stack([rad0 * np.cos(th0), rad0 * np.sin(th0), rad1 * np.cos(th1), rad1 * np.sin(th1)],
                 axis=1).reshape(-1)
    return z[:n].astype(np.float32)


# Random123 known-answer vectors for philox4x32_10 (kat_vectors: ctr, key, expected)
KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]
