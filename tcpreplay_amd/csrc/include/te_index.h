/*
 * te_index.h -- the device record index (te_index.hip): the arguments of its single pass,
 * shared with the C host (te_api.c).
 */
#ifndef TE_INDEX_H
#define TE_INDEX_H
#include <stdint.h>
#include "te_kernels.h"

#ifndef TE_IDX_S
#define TE_IDX_S 80     /* sub-window bytes per lane: a wave stages 64 x TE_IDX_S bytes */
#endif
#ifndef TE_IDX_OL
#define TE_IDX_OL 7     /* of which the first TE_IDX_OL sub-windows are the previous window's
                           last bytes (they establish the chain entering the window) */
#endif
#define IDX_NONE 0xffffffffffffffffull
/* how the chain ends in a window (w_flags) */
#define IDX_STOP 1u   /* oversize record: libpcap stops (walk_stop 1) */
#define IDX_ERROR 2u  /* len > 262144: the reference's error (walk_stop 2) */
#define IDX_END 4u    /* a truncated record or the bytes ran out */
#define IDX_ZERO 8u   /* a record with caplen 0 */
#define IDX_OVF 16u   /* the window's tiles or records did not fit tile_cap / rec_cap */
/* totals[] */
#define IDX_T_RECS 0
#define IDX_T_TILES 1
#define IDX_T_BYTES 2   /* sum of 16 + caplen + growth (the output bound) */
#define IDX_T_SCRATCH 3
#define IDX_T_BAD 4     /* a window's guess was not where the chain is: use the host walk */
#define IDX_T_WINDOWS 5 /* windows up to the chain's end */
#define IDX_T_STOP 6    /* IDX_STOP / IDX_ERROR / IDX_END, or 0 */
#define IDX_T_END 7     /* offset of the first record not taken */
#define IDX_T_ZERO 8
#define IDX_T_ERR_REC 9 /* the record with the len error, or ~0 */
#define IDX_T_OVERFLOW 10 /* the tiles or records outgrew tile_cap / rec_cap */
#define IDX_T_BADWIN 11 /* diagnostics: the first window whose guess missed the chain */
#define IDX_T__N 12

/* the per-launch words the pass needs zeroed, at the start of its workspace:
   ticket, the first stop / bad / zero-caplen / overflow windows (complemented), timeouts
   (u32 each), scratch counter (u64) */
#define IDX_WS_WORDS 64
#define IDX_WS_BYTES(nwin) (IDX_WS_WORDS + 8ull * (nwin) /* state */)
/* per-window records the finishing wave reads (not zeroed) */
#define IDX_WIN_BYTES(nwin) (8ull * 4 * (nwin) /* entry, exit, pfx, err */ + 4ull * (nwin) /* flags */)

#ifdef __cplusplus
extern "C" {
#endif
typedef struct {
    const uint8_t *img; /* device: the pcap image (its records from file offset `entry` on) */
    uint64_t len;       /* bytes of the image (record bytes end here) */
    uint64_t entry;     /* image offset of the first record (24 for a whole capture) ... */
    const uint64_t *entry_ptr; /* ... or, when set, *entry_ptr - entry_sub, read on the device
                                  (a pipeline chunk: where the previous chunk's chain ended) */
    uint64_t entry_sub;
    uint64_t base;      /* the window grid's origin: 16-aligned, <= the first record */
    uint64_t limit;     /* records starting here or later are not this image's (<= len) */
    int32_t sw, nsec;
    uint32_t nwin;      /* windows of te_index_window_bytes() from entry & ~15 */
    uint32_t budget, max_pkts, growth; /* the wave-lane tile cut (walk_range) */
    /* zeroed per launch (IDX_WS_BYTES) */
    uint32_t *ticket, *stop_win_c, *bad_win_c, *zero_win_c, *ovf_win_c, *timeouts; /* (~first window) */
    uint64_t *scratch_ctr;
    uint64_t *state;    /* nwin look-back granules */
    /* per window (IDX_WIN_BYTES) */
    uint64_t *w_entry, *w_exit, *w_pfx, *w_err;
    uint32_t *w_flags;
    uint64_t *totals;   /* IDX_T__N words */
    /* the batch's index */
    te_tile_t *tiles;
    uint16_t *pkt_rel;
    uint64_t tile_cap, rec_cap;
} IdxArgs;
/* bytes of a window */
uint32_t te_index_window_bytes(void);
/* the single pass (the workspace words zeroed by the caller first) */
int te_launch_index(const IdxArgs *a, void *stream);
#ifdef __cplusplus
}
#endif
#endif
