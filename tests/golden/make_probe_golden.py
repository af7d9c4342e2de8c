#!/usr/bin/env python3
"""Generate the row pre-probe fixture.

Run HERE (the build container), where /root/reference exists:

    make -C oracle ref && python tests/golden/make_probe_golden.py

Everything expected in the fixture comes from the REFERENCE's own code
(oracle/_ref/libref_shf.so = /root/reference/src/murmurhash3.c + shf.c, plus
oracle/ref_harness.c and oracle/ref_export.c):
  * ref_hash:  shf_make_hash() of every key (src/shf.c:450-462);
  * ref_uid:   shf_uid after the reference's own shf_get_key_val_addr() of
               every key (src/shf.c:1032 -> shf_find_key_internal, :886-936),
               0xffffffff when the key is not in the store;
  * tab_slot / rows: the store's tab map and rows after the reference's own
               shf_put_key_val() of keys [0, n_put) (src/shf.c:780-878),
               exported by ref_export_rows() in the row-index layout of
               include/shf_hash_batch.h.

Keys: 6,000 whose window is 0 (so window 0's rows overflow and the reference
parts tab 0 several times, src/shf.c:722-779), 3,000 spread over all windows,
then 1,000 more that are never put (absent lookups). 16 bytes each, from
sharedhashfile_amd.keygen.splitmix_bytes.

Output: tests/golden/probe_fixture.npz (data only).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle.oracle_py import reference_lib, reference_probe_fixture  # noqa: E402
from sharedhashfile_amd.keygen import splitmix_bytes  # noqa: E402

N_WIN0, N_OTHER, N_ABSENT = 6000, 3000, 1000


def main():
    lib = reference_lib()
    if lib is None:
        raise SystemExit("build oracle/_ref first: make -C oracle ref")
    cand = np.frombuffer(splitmix_bytes(2_000_000 * 16, 0x5EED0F3), dtype=np.uint8).reshape(-1, 16)
    off = np.arange(cand.shape[0] + 1, dtype=np.uint64) * 16
    h = np.empty((cand.shape[0], 2), dtype=np.uint64)
    lib.ref_hash_var(cand.ctypes.data, off.ctypes.data, cand.shape[0], h.ctypes.data)
    win0 = (h[:, 0] & 0xFF) == 0
    keys = np.concatenate([cand[win0][:N_WIN0], cand[~win0][: N_OTHER + N_ABSENT]])
    hashes = np.concatenate([h[win0][:N_WIN0], h[~win0][: N_OTHER + N_ABSENT]])
    assert keys.shape[0] == N_WIN0 + N_OTHER + N_ABSENT
    koff = np.arange(keys.shape[0] + 1, dtype=np.uint64) * 16
    n_put = N_WIN0 + N_OTHER
    uids, tab_slot, rows = reference_probe_fixture(keys, koff, n_put)
    assert (uids[:n_put] != 0xFFFFFFFF).all() and (uids[n_put:] == 0xFFFFFFFF).all()
    tabs_win0 = len(set((tab_slot[:2048] & 0x7FF).tolist()))
    assert tabs_win0 > 1, "window 0 was expected to part"
    out = os.path.join(HERE, "probe_fixture.npz")
    np.savez_compressed(out, keys=keys, n_put=np.uint64(n_put), ref_hash=hashes, ref_uid=uids, tab_slot=tab_slot,
                        rows=rows)
    print("wrote %s: %d keys, %d slots, window 0 parted into %d tabs (%d bytes)" % (
        out, keys.shape[0], rows.size // 65536, tabs_win0, os.path.getsize(out)))


if __name__ == "__main__":
    main()
