"""Decode-step model of the 3-D brick decoder's rows (CPU, oracle): code lengths of the (0, 0)
row of each 8 x 8 yz tile against the others, and quarters of kF = 4 Tab4 steps per 256-symbol
row (two symbols per step when both codes fit 12 bits; codes over 16 bits stop the lane for the
rest of its quarter, then one long step)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import pyoracle as po  # noqa: E402
from cusz_amd import datagen  # noqa: E402


def quarters(L):
    i, q, longs, steps = 0, 0, 0, 0
    n = len(L)
    while i < n:
        q += 1
        stalled = False
        for _ in range(4):
            if i >= n:
                break
            if L[i] > 16:
                stalled = True
                break
            steps += 1
            if L[i] <= 12 and i + 1 < n and L[i] + L[i + 1] <= 12:
                i += 2
            else:
                i += 1
        if stalled:
            longs += 1
            steps += 1
            i += 1
    return q, longs, steps


def main():
    dims = (256, 128, 128)
    d = datagen.smooth3d_np(dims)
    eb = 1e-4 * float(d.max() - d.min())
    codes, *_ = po.lorenzo_c(d, dims, eb)
    codes = np.asarray(codes).reshape(dims[2], dims[1], dims[0])
    hist = po.histogram(codes.ravel())
    L = po.huffman_lengths(hist)
    for name, sel in (("(0,0)", lambda y, z: y % 8 == 0 and z % 8 == 0), ("y>0,z=0", lambda y, z: y % 8 and z % 8 == 0),
                      ("y=0,z>0", lambda y, z: y % 8 == 0 and z % 8), ("inner", lambda y, z: y % 8 and z % 8)):
        qs, ls, ss, l12, l16 = [], [], [], [], []
        for z in range(dims[2]):
            for y in range(dims[1]):
                if not sel(y, z):
                    continue
                row = L[codes[z, y, :]]
                q, lg, st = quarters(row)
                qs.append(q), ls.append(lg), ss.append(st)
                l12.append(int((row > 12).sum())), l16.append(int((row > 16).sum()))
        print(f"{name:8s} rows {len(qs):5d}  quarters mean {np.mean(qs):6.1f} max {max(qs):4d}  steps {np.mean(ss):6.1f}  "
              f"codes>12 {np.mean(l12):5.1f}  >16 {np.mean(l16):5.1f}  long quarters {np.mean(ls):5.1f}")


if __name__ == "__main__":
    main()
