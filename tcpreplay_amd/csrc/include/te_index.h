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
#define TE_IDX_OL 2     /* of which the first TE_IDX_OL sub-windows are the previous window's
                           last bytes (they establish the chain entering the window) */
#endif
#define IDX_NONE 0xffffffffffffffffull
/* how the chain ends in a window (w_flags) */
#define IDX_STOP 1u   /* oversize record: libpcap stops (walk_stop 1) */
#define IDX_ERROR 2u  /* len > 262144, len 0 or caplen 0: safe_pcap_next exits (walk_stop 2) */
#define IDX_END 4u    /* a truncated record or the bytes ran out */
#define IDX_TRIM 8u   /* a record with len < caplen: safe_pcap_next trims it (utils.c:159-162) */
/* totals[] */
#define IDX_T_RECS 0
#define IDX_T_TILES 1
#define IDX_T_BYTES 2   /* sum of 16 + caplen + growth (the output bound) */
#define IDX_T_SCRATCH 3
#define IDX_T_BAD 4     /* a window's guess was not where the chain is: use the host walk */
#define IDX_T_WINDOWS 5 /* windows up to the chain's end */
#define IDX_T_STOP 6    /* IDX_STOP / IDX_ERROR / IDX_END, or 0 */
#define IDX_T_END 7     /* offset of the first record not taken */
#define IDX_T_TRIM 8
#define IDX_T_ERR_REC 9 /* the record with the len error, or ~0 */
#define IDX_T_OVERFLOW 10 /* the tiles or records outgrew tile_cap / rec_cap */
#define IDX_T_BADWIN 11 /* diagnostics: the first window whose guess missed the chain */
#define IDX_T__N 12

/* records starting in one window, at most (a record is at least its 16-byte header) */
#define IDX_MAXR (64 * TE_IDX_S / 16)
/* the index's device workspace for nwin windows: per window its facts (entry, exit, flags,
   records|tiles, scratch bytes) and prefixes (records|tiles, scratch), the totals, and the
   count pass's cut (record offsets in their tiles, tile starts) for the write pass */
#define IDX_SB 1024        /* windows a block of the scan's first level takes */
#define IDX_PART_BYTES 32  /* such a block's record */
#define IDX_WS_BYTES(nwin) (8ull * 7 * (nwin) + 4ull * ((nwin) + 1) + 8ull * (IDX_T__N + 2) + \
                            IDX_PART_BYTES * ((nwin) / IDX_SB + 2) + (2ull + 8ull) * IDX_MAXR * (nwin) + 64)

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
    /* per window (IDX_WS_BYTES) */
    uint64_t *w_entry, *w_exit, *w_agg, *w_scr, *w_pfx, *w_sbase;
    int64_t *w_prev;    /* the nearest earlier window with a record, within its scan block */
    void *parts;        /* the part blocks' totals, then their prefixes (IDX_PART_BYTES each) */
    uint32_t *w_flags;
    uint16_t *t_prel;   /* IDX_MAXR a window: each record's offset in its tile */
    uint32_t *t_tile;   /* IDX_MAXR pairs a window: {first offset from the window, first | npkt << 16} */
    uint64_t *totals;   /* IDX_T__N words */
    /* the batch's index */
    te_tile_t *tiles;
    uint16_t *pkt_rel;
    uint64_t tile_cap, rec_cap;
} IdxArgs;
/* bytes of a window */
uint32_t te_index_window_bytes(void);
/* count, scan and write (nothing to zero first) */
int te_launch_index(const IdxArgs *a, void *stream);
#ifdef __cplusplus
}
#endif
#endif
