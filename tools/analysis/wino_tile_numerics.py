"""Winograd tile size vs the 1e-5 flow contract (dev analysis, CPU, numpy).

Emulates the wx3 arithmetic -- f32 input transform, V split into f16 (hi, lo), U*2^k split into
f16 pairs from float64, three f16 x f16 products accumulated in f32, f32 output transform --
for F(2x2,3x3) (the kernel) and F(4x4,3x3), and reports the max error scaled as in
tests/test_gpu_wx3.py (|y - ref| / max(|ref|, 1)) against a float64 direct 3x3 correlation.
Variant "f64 transforms": V and the output transform in float64 (only the split, the products
and the f32 accumulation rounded) -- the floor no cheaper transform arithmetic can beat.

usage: python tools/analysis/wino_tile_numerics.py
"""
import numpy as np

f16, f32, f64 = np.float16, np.float32, np.float64


def mats(m):
    if m == 2:
        BT = [[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]]
        G = [[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]]
        AT = [[1, 1, 1, 0], [0, 1, -1, -1]]
    else:
        BT = [[4, 0, -5, 0, 1, 0], [0, -4, -4, 1, 1, 0], [0, 4, -4, -1, 1, 0],
              [0, -2, -1, 2, 1, 0], [0, 2, -1, -2, 1, 0], [0, 4, 0, -5, 0, 1]]
        G = [[1 / 4, 0, 0], [-1 / 6, -1 / 6, -1 / 6], [-1 / 6, 1 / 6, -1 / 6],
             [1 / 24, 1 / 12, 1 / 6], [1 / 24, -1 / 12, 1 / 6], [0, 0, 1]]
        AT = [[1, 1, 1, 1, 1, 0], [0, 1, -1, 2, -2, 0], [0, 1, 1, 4, 4, 0], [0, 1, -1, 8, -8, 1]]
    return np.array(BT, f64), np.array(G, f64), np.array(AT, f64)


def run(m, C, T, N=8, exact_transforms=False, seed=0):
    rng = np.random.default_rng(seed)
    a = m + 2
    BT, G, AT = mats(m)
    d = rng.standard_normal((T, C, a, a)).astype(f32)
    w = rng.standard_normal((N, C, 3, 3)) / np.sqrt(9 * C)
    ref = np.zeros((T, N, m, m))
    for y in range(m):
        for x in range(m):
            ref[:, :, y, x] = np.einsum('tcij,ncij->tn', d[:, :, y:y + 3, x:x + 3].astype(f64), w)
    U = np.einsum('ai,ncij,bj->ncab', G, w, G)
    k = np.floor(np.log2(2 ** 15 / np.abs(U).max(axis=(1, 2, 3), keepdims=True)))
    Us = U * 2.0 ** k
    Uh = Us.astype(f16)
    Ul = (Us - Uh.astype(f64)).astype(f16)
    tdt = f64 if exact_transforms else f32
    V = np.einsum('ai,tcij->tcaj', BT.astype(tdt), d.astype(tdt)).astype(tdt)
    V = np.einsum('tcaj,bj->tcab', V, BT.astype(tdt)).astype(f32)
    Vh = V.astype(f16)
    Vl = (V - Vh.astype(f32)).astype(f16)
    prod = lambda p, q: np.einsum('tcab,ncab->tnab', p.astype(f32), q.astype(f32), dtype=f32)  # noqa
    M = (prod(Vh, Uh) + prod(Vh, Ul) + prod(Vl, Uh)).astype(f32)
    M = (M * (2.0 ** -k).reshape(1, N, 1, 1)).astype(tdt)
    Y = np.einsum('ia,tnab->tnib', AT.astype(tdt), M).astype(tdt)
    Y = np.einsum('tnib,jb->tnij', Y, AT.astype(tdt)).astype(f32)
    return (np.abs(Y - ref) / np.maximum(np.abs(ref), 1.0)).max()


if __name__ == "__main__":
    for C in (52, 496):
        for m in (2, 4):
            T = 3000 if m == 2 else 1000
            print(f"c={C:3d} F({m}x{m},3x3): f32 transforms {run(m, C, T):.2e}   "
                  f"f64 transforms {run(m, C, T, exact_transforms=True):.2e}")
