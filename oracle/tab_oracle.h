/*
 * TEST INFRASTRUCTURE ONLY -- CPU oracle of the tab part / shrink copy
 * (SURVEY.md §8 f4). Only tests/ may load it, and only as the checker; the
 * product (sharedhashfile_amd/, include/shf_hash_batch.h) never links it.
 *
 * Restates, for one tab image (the bytes of a tab file: SHF_TAB_MMAP header,
 * 512 rows of 16 refs, key,value data; /root/reference/src/shf.private.h:48-68):
 *   shf_tab_part()   /root/reference/src/shf.c:722-779 -- every ref whose tab2
 *                    the window's (already redirected) map sends to tab_new is
 *                    copied to a fresh tab (SHF_TAB_REF_COPY, :633-651, which
 *                    appends with SHF_TAB_APPEND, :545-610), then the old tab is
 *   shf_tab_shrink() /root/reference/src/shf.c:678-720 -- re-created and every
 *                    remaining ref copied into it, in row/ref order.
 * Both outputs are fresh tabs filled by appends in row/ref order, so one pass
 * produces both. Pinned by tests/test_tab_oracle.py against tab files the
 * reference itself wrote (oracle/ref_export.c ref_part_capture(), fixture
 * tests/golden/tab_part_fixture.npz).
 */
#ifndef SHF_TAB_ORACLE_H
#define SHF_TAB_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_TAB_NONE 0xffffu

/* src: src_len bytes of a tab image. map: the window's 2048 tab2 -> tab entries
 * after shf_tab_part()'s redirect (tab_new == ORACLE_TAB_NONE: shrink only, no
 * ref moves). fixed != 0: a fixed-length store (keys key_len, values val_len
 * bytes, no length words). factor: the reference's data-needed factor.
 * keep_type / move_type: the data-type byte written at the start of each copied
 * record. SHF_TAB_APPEND sets key_type and val_type of a stack SHF_DATA_TYPE
 * and never its `extended` bit (shf.c:593-596), so the reference writes 0x3e
 * or 0xbe depending on its stack: its build writes 0xbe in shf_tab_part()'s
 * copies and 0x3e in shf_tab_shrink()'s (the values its own tab files show).
 * keep / move: zero-filled output images of keep_cap / move_cap bytes (move may
 * be NULL for a shrink). Returns 0, or -1 if an output does not fit. */
int oracle_tab_split(const uint8_t *src, uint64_t src_len, const uint16_t *map, uint32_t tab_new, int fixed,
                     uint32_t key_len, uint32_t val_len, uint32_t factor, uint32_t keep_type, uint32_t move_type,
                     uint8_t *keep, uint64_t keep_cap, uint8_t *move, uint64_t move_cap);

/* shf_tab_part()'s redirect of a window's map (shf.c:683-692): of the tab2
 * entries naming tab_old, every second one (the 2nd, 4th, ...) now names tab_new. */
void oracle_tab_part_redirect(uint16_t *map, uint32_t tab_old, uint32_t tab_new);

#ifdef __cplusplus
}
#endif
#endif
