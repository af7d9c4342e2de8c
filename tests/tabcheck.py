"""Comparison of a computed tab image (CPU oracle or GPU) with the tab file the
reference itself wrote (oracle/ref_export.c ref_part_capture()), for the f4
tab part / shrink copy.

The put that parted the tab (shf.c:829-834) then put its own key into one of
the two tabs (shf.c:809-827 after `goto SHF_NEED_NEW_TAB_AFTER_PARTING`): that
tab's file holds, beyond the part's result, one more record at the end of its
data and one more ref. `expect_tab` checks the computed image against the file
with exactly that difference, everything else byte for byte.
"""
import numpy as np

TAB_HDR = 24
TAB_DATA = TAB_HDR + 512 * 16 * 8  # offsetof(SHF_TAB_MMAP, data)
PAGE = 4096


def hdr(img):
    return [int(x) for x in np.frombuffer(img[:TAB_HDR].tobytes(), dtype=np.uint32)]


def mod_page(b):
    return ((b - 1) // PAGE + 1) * PAGE


def put_slot(cap):
    """(tab the put key went to, row, ref) from the capture's uid (shf.private.h:170-178)."""
    uid = cap["uid"]
    tab2 = (uid >> 8) & 0x7FF
    return int(cap["map_after"][tab2]), (uid >> 19) & 0x1FF, uid >> 28


def put_record_len(cap, key_len):
    if cap["fixed"]:
        return 1 + cap["fixed_key_len"] + cap["fixed_val_len"]
    return 1 + 4 + key_len + 4 + 8  # value: the 8-byte key index (ref_part_capture)


def expect_tab(got, ref, slot=None, rec_len=0, factor=1):
    """got: computed image (zero beyond what it wrote); ref: the reference's file
    after the put; slot: (row, ref) of the put's key if it went to this tab."""
    got = np.asarray(got, dtype=np.uint8)
    ref = np.asarray(ref, dtype=np.uint8)
    g = hdr(got)
    r = hdr(ref)
    used = g[1]
    assert used >= TAB_DATA and g[3] == 0 and g[4] == 0 and g[5] == used - TAB_DATA, g
    rows_g = got[TAB_HDR:TAB_DATA].view(np.uint32).reshape(512, 16, 2).copy()
    rows_r = ref[TAB_HDR:TAB_DATA].view(np.uint32).reshape(512, 16, 2).copy()
    if slot is None:
        assert g == r, (g, r)
        assert g[0] == ref.size
    else:
        row, k = slot
        assert rows_g[row, k].tolist() == [0, 0], "the put's slot is empty in the part's result"
        assert rows_r[row, k, 1] == used, "the put's record follows the part's data"
        rows_r[row, k] = 0
        size = g[0] + 0
        if rec_len > size - used:
            size = mod_page(size + rec_len * factor)
        assert r == [size, used + rec_len, g[2] + 1, 0, 0, g[5] + rec_len], (g, r, rec_len)
        assert size == ref.size
    assert np.array_equal(rows_g, rows_r)
    assert np.array_equal(got[TAB_DATA:used], ref[TAB_DATA:used])
    assert not got[used:].any()


def observed_types(cap):
    """(keep_type, move_type): the SHF_DATA_TYPE byte the reference wrote at the
    records it copied into the shrunk old tab and the new tab. Its `extended`
    bit is never initialised by SHF_TAB_APPEND (shf.c:593-596), so the byte is
    whatever the reference's stack held (0x3e or 0xbe; oracle/tab_oracle.h);
    the copy takes it as a parameter."""
    tab, row, k = put_slot(cap)
    out = []
    for img, t in ((cap["old"], cap["tab_old"]), (cap["new"], cap["tab_new"])):
        rows = np.asarray(img[TAB_HDR:TAB_DATA]).view(np.uint32).reshape(512, 16, 2).copy()
        if t == tab:
            rows[row, k] = 0  # the put's own record (shf_put_key_val's append)
        pos = rows[:, :, 1][rows[:, :, 1] != 0]
        vals = np.unique(np.asarray(img)[pos]) if pos.size else np.array([0x3E], np.uint8)
        assert vals.size == 1, vals  # one byte per copy loop
        out.append(int(vals[0]))
    return tuple(out)


def check_capture(cap, keep, move, put_key_len):
    """keep / move: the computed shrunk old tab and new tab for capture `cap`."""
    tab, row, k = put_slot(cap)
    rec = put_record_len(cap, put_key_len)
    expect_tab(keep, cap["old"], (row, k) if tab == cap["tab_old"] else None, rec, cap["factor"])
    expect_tab(move, cap["new"], (row, k) if tab == cap["tab_new"] else None, rec, cap["factor"])
