#!/usr/bin/env python3
"""Write tests/golden/pms/tiny_v2.pms and its expected tables (tiny_v2_tables.npz).

The file is hand-made in RASR's mixture-set text format (src/Mm/MixtureSet.cc:142-168)
with the number spellings a real file may hold; the expected tables come from the
std::istream restatement of MixtureSet::read (oracle/pms_istream.cc), i.e. the same
libstdc++ extraction the reference performs.  The reference holds no .pms files of
its own to use instead.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import pms  # noqa: E402

TEXT = """#Version: 2.0
#CovarianceType: DiagonalCovariance
4 4 6 5 2
2 0 -0.693147 1 -0.693147
3 2 -1.09861 3 -1.09861 4 -1.0986122886681098
0
1 5 0
0 0
1 0
2 1
3 1
4 1
4 1
4 0.5 -1.25 2.0000001 1e-07
4 +3.25 -0 .125 6.
4 1E2 -2.5e-1 0.1 0.2
4 3.4028234e38 -1.17549435e-38 1.4e-45 0.333333333333333333333
4 -7 7 -7 7
 4 1 1 2.5 1 0.75 2 4 0.25
 4 0.5 1 0.5 1 0.5 1 1.5 1
"""


def main():
    out = os.path.join(ROOT, "tests", "golden", "pms")
    path = os.path.join(out, "tiny_v2.pms")
    with open(path, "w") as f:
        f.write(TEXT)
    rc, t = pms.pms_read(path)
    assert rc == pms.OK, rc
    np.savez(os.path.join(out, "tiny_v2_tables.npz"), **t)
    print("wrote", path, {k: v.shape for k, v in t.items()})


if __name__ == "__main__":
    main()
