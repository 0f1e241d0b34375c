"""Compare two .npz dumps array by array: bitwise-equal count and max abs difference."""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
bad = 0
for k in a.files:
    x, y = a[k], b[k]
    same = np.array_equal(x, y)
    bad += not same
    print(("OK  " if same else "DIFF"), k, x.shape, float(np.abs(x - y).max()) if x.size else 0)
sys.exit(1 if bad else 0)
