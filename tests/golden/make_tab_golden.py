"""Generate tests/golden/tab_part_fixture.npz: shf_tab_part() (+ its
shf_tab_shrink()) done by the reference itself.

Keys that all land in window 0 are put one by one into a fresh store by the
reference's own shf_put_key_val(), compiled from /root/reference/src into
oracle/_ref/libref_shf.so; oracle/ref_export.c ref_part_capture() copies the
parted tab's file before the put and both tab files after it, and the
window's tab2 -> tab map before and after. Two captures:

  c0  variable-length keys 8..40 B, 8-B values, data-needed factor 1
  c1  fixed-length store (16-B keys, 8-B values), data-needed factor 3

Run (in the build container, where /root/reference exists):
    python tests/golden/make_tab_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.oracle_py import Oracle, reference_part_capture  # noqa: E402
from sharedhashfile_amd.keygen import splitmix_bytes, splitmix_lengths  # noqa: E402

CASES = [  # (name, key length lo, hi, fixed key len, fixed val len, factor, stream)
    ("c0", 8, 40, 0, 0, 1, 99),
    ("c1", 16, 16, 16, 8, 3, 107),
]


def window0_keys(o, n, lo, hi, stream):
    """Keys (packed bytes + offsets) whose shf_make_hash() window is 0."""
    lens = splitmix_lengths(n, lo, hi, stream)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    data = np.frombuffer(splitmix_bytes(int(off[-1]), stream + 1), dtype=np.uint8)
    h = o.hash_var(data, off)
    sel = np.nonzero((h[:, 0] & np.uint64(0xFF)) == 0)[0]
    keys = [data[int(off[i]):int(off[i + 1])] for i in sel]
    o2 = np.zeros(len(keys) + 1, np.uint64)
    o2[1:] = np.cumsum([k.size for k in keys])
    return np.concatenate(keys), o2


def main():
    o = Oracle()
    out = {}
    for name, lo, hi, fk, fv, fac, stream in CASES:
        data, off = window0_keys(o, 3_000_000, lo, hi, stream)
        cap = reference_part_capture(data, off, fixed_key_len=fk, fixed_val_len=fv, factor=fac, max_caps=1)[0]
        k = cap["key"]
        out[name + "_before"] = cap["before"]
        out[name + "_old"] = cap["old"]
        out[name + "_new"] = cap["new"]
        out[name + "_map_before"] = cap["map_before"]
        out[name + "_map_after"] = cap["map_after"]
        out[name + "_meta"] = np.array([cap["win"], cap["tab_old"], cap["tab_new"], cap["uid"], k, cap["fixed"],
                                        cap["fixed_key_len"], cap["fixed_val_len"], cap["factor"],
                                        int(off[k + 1] - off[k])], dtype=np.int64)
    path = os.path.join(HERE, "tab_part_fixture.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
