/*
 * te_index.h -- the device record index (te_index.hip): the arguments of its three
 * passes (count, scan, write), shared with the C host (te_api.c).
 */
#ifndef TE_INDEX_H
#define TE_INDEX_H
#include <stdint.h>
#include "te_kernels.h"

#define IDX_NONE 0xffffffffffffffffull
/* how the chain ends in a window (w_flags) */
#define IDX_STOP 1u   /* oversize record: libpcap stops (walk_stop 1) */
#define IDX_ERROR 2u  /* len > 262144: the reference's error (walk_stop 2) */
#define IDX_END 4u    /* a truncated record or the bytes ran out */
#define IDX_ZERO 8u   /* a record with caplen 0 */
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
#define IDX_T__N 10

#ifdef __cplusplus
extern "C" {
#endif
typedef struct {
    const uint8_t *img; /* device: the pcap image (records from offset 24) */
    uint64_t len;
    int32_t sw, nsec;
    uint64_t W;         /* window bytes (a multiple of 64) */
    uint32_t nwin;
    uint32_t budget, max_pkts, growth; /* the wave-lane tile cut (walk_range) */
    /* per window (count pass -> scan) */
    uint64_t *w_entry, *w_exit, *w_recbytes, *w_scratch;
    uint32_t *w_nrec, *w_ntile, *w_flags, *w_err;
    /* per window bases (scan -> write pass) */
    uint64_t *p_base, *t_base, *s_base;
    uint64_t *totals;   /* IDX_T__N words */
    /* the batch's index (write pass) */
    te_tile_t *tiles;
    uint16_t *pkt_rel;
} IdxArgs;
/* pass 0: count, 1: scan, 2: write */
int te_launch_index(const IdxArgs *a, int pass, void *stream);
#ifdef __cplusplus
}
#endif
#endif
