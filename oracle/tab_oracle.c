/* TEST INFRASTRUCTURE ONLY -- see tab_oracle.h. */
#include "tab_oracle.h"

#include <string.h>

#define TAB_HDR 24u                      /* 6 x u32: tab_size, tab_used, tab_refs_used, tab_data_free_pos,
                                            tab_data_free, tab_data_used (shf.private.h:59-65) */
#define TAB_ROWS 512u                    /* SHF_ROWS_PER_TAB */
#define TAB_REFS 16u                     /* SHF_REFS_PER_ROW */
#define TAB_DATA (TAB_HDR + TAB_ROWS * TAB_REFS * 8u) /* offsetof(SHF_TAB_MMAP, data) = 65560 */
#define PAGE 4096u                       /* SHF_SIZE_PAGE */

static uint32_t get32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static void put32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
static uint64_t mod_page(uint64_t b) { return ((b - 1) / PAGE + 1) * PAGE; } /* SHF_MOD_PAGE, shf.defines.h:76 */

typedef struct {
    uint8_t *img;
    uint64_t cap;
    uint64_t size, used;
    uint32_t refs, data_used;
    uint8_t type; /* SHF_DATA_TYPE byte of the copies (see tab_oracle.h) */
} tab_out;

/* A tab as shf_tab_create() + SHF_GET_TAB_MMAP leave it (shf.c:358-373, :496-501):
 * file size MOD_PAGE(sizeof(SHF_TAB_MMAP)), tab_used = offsetof(data). */
static void out_init(tab_out *o, uint8_t *img, uint64_t cap, uint32_t type)
{
    o->type = (uint8_t)type;
    o->img = img;
    o->cap = cap;
    o->size = mod_page(TAB_DATA);
    o->used = TAB_DATA;
    o->refs = 0;
    o->data_used = 0;
}

/* SHF_TAB_APPEND on a tab with no deleted data (no free-list reuse): grow the
 * tab if the record does not fit (shf.c:562-565), copy it at tab_used with the
 * output's data-type byte (:593-606). Returns the record's pos, or 0 if it
 * cannot fit cap. */
static uint64_t out_append(tab_out *o, const uint8_t *rec, uint32_t len, uint32_t factor)
{
    if ((uint64_t)len > o->size - o->used) o->size = mod_page(o->size + (uint64_t)len * factor);
    if (o->used + len > o->cap) return 0;
    const uint64_t pos = o->used;
    memcpy(o->img + pos, rec, len);
    o->img[pos] = o->type;
    o->used += len;
    o->refs += 1;
    o->data_used += len;
    return pos;
}

static void out_header(tab_out *o)
{
    put32(o->img + 0, (uint32_t)o->size);
    put32(o->img + 4, (uint32_t)o->used);
    put32(o->img + 8, o->refs);
    put32(o->img + 12, 0);
    put32(o->img + 16, 0);
    put32(o->img + 20, o->data_used);
}

int oracle_tab_split(const uint8_t *src, uint64_t src_len, const uint16_t *map, uint32_t tab_new, int fixed,
                     uint32_t key_len, uint32_t val_len, uint32_t factor, uint32_t keep_type, uint32_t move_type,
                     uint8_t *keep, uint64_t keep_cap, uint8_t *move, uint64_t move_cap)
{
    const uint32_t len_len = fixed ? 0u : 4u; /* shf.c:674: sizeof(fixed_key_len) unless fixed */
    tab_out k, m;
    if (keep_cap < TAB_DATA || (move && move_cap < TAB_DATA) || src_len < TAB_DATA) return -1;
    out_init(&k, keep, keep_cap, keep_type);
    if (move) out_init(&m, move, move_cap, move_type);
    for (uint32_t row = 0; row < TAB_ROWS; ++row) {
        for (uint32_t ref = 0; ref < TAB_REFS; ++ref) {
            const uint8_t *r = src + TAB_HDR + (row * TAB_REFS + ref) * 8u;
            const uint32_t w0 = get32(r), pos = get32(r + 4); /* {tab:11 | rnd:21}, pos (shf.private.h:48-52) */
            if (!pos) continue;                              /* ref unused */
            const uint32_t tab2 = w0 & 0x7ffu;
            const int moves = move && tab_new != ORACLE_TAB_NONE && map[tab2] == tab_new; /* shf.c:765-767 */
            /* SHF_TAB_REF_COPY's lengths (shf.c:636-637) */
            const uint32_t kl = fixed ? key_len : get32(src + pos + 1);
            const uint32_t vl = fixed ? val_len : get32(src + pos + 1 + len_len + kl);
            const uint32_t len = 1u + len_len + kl + len_len + vl;
            if (pos + (uint64_t)len > src_len) return -1;
            tab_out *o = moves ? &m : &k;
            const uint64_t np = out_append(o, src + pos, len, factor ? factor : 1u);
            if (!np) return -1;
            /* SHF_TAB_APPEND counted the ref (shf.c:608); SHF_TAB_REF_COPY counts it
             * again (:651): a copied tab's tab_refs_used is twice its refs in the
             * reference, restated as is */
            o->refs += 1;
            uint8_t *d = o->img + TAB_HDR + (row * TAB_REFS + ref) * 8u; /* same row and ref (shf.c:648-650) */
            put32(d, w0);
            put32(d + 4, (uint32_t)np);
        }
    }
    out_header(&k);
    if (move) out_header(&m);
    return 0;
}

void oracle_tab_part_redirect(uint16_t *map, uint32_t tab_old, uint32_t tab_new)
{
    uint32_t sw = 0;
    for (uint32_t tab2 = 0; tab2 < 2048u; ++tab2) {
        if (map[tab2] == tab_old) {
            map[tab2] = (uint16_t)(sw ? tab_new : tab_old);
            sw = !sw;
        }
    }
}
