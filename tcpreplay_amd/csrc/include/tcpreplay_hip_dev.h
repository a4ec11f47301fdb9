/*
 * tcpreplay_hip_dev.h -- one replay pass as the gfx950 kernels take it
 * (tcpreplay_kernels.hip), shared with the C host (tr_api.c).
 */
#ifndef TCPREPLAY_HIP_DEV_H
#define TCPREPLAY_HIP_DEV_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* the --include / --exclude packet list (parse_list, src/common/list.c:61-130): ranges
   [min, max] with check_list's (:139-156) open ends -- min 0: up to max, max 0: from min */
typedef struct {
    uint64_t *rng;        /* host: n pairs {min, max} */
    uint32_t n;
    int32_t exclude;      /* --exclude (else --include) */
} tr_list_t;
/* 0, or -1 with the reference's message in err ("Unable to parse include/exclude rule") */
int tr_list_parse(tr_list_t *l, const char *arg, int exclude, char *err, size_t errlen);
void tr_list_free(tr_list_t *l);

typedef struct {
    const uint8_t *img;   /* device capture image (records at off[j]) */
    uint8_t *cache;       /* -K: the device copy edited from pass to pass, else NULL */
    int32_t cached;       /* fast_edit_packet's `cached` arithmetic (the -K passes after the first) */
    const uint64_t *list; /* device: the packet list's {min, max} pairs (packet number = j + 1), or NULL */
    uint32_t nlist;
    int32_t exclude;
    uint64_t *nfail;      /* device word: records whose edit failed (atomic adds), or NULL */
    const uint64_t *off;  /* record offsets */
    uint64_t n;
    int32_t swapped, nsec;
    int32_t edit;         /* this pass edits (unique_iteration advanced, send_packets.c:477) */
    uint64_t iteration;   /* unique_iteration - 1 */
    uint64_t *size;       /* per record: output bytes (0: edit failed, not sent) */
    uint64_t *pos;        /* per record: output offset within the pass */
    void *patch;          /* uint4 per record: {at_s, src, at_d, dst} */
    uint8_t *out;         /* the pass's output */
    int32_t mark_only;    /* only the sizes and patches (tcpreplay-edit places the records itself) */
} TrPass;
size_t tr_scan_temp_bytes(uint64_t n);
/* the list as a tcpprep v04 cache body for n records: a listed-out record NOSEND (bits 00),
   the rest C2S (bits 11) -- the edit batch then leaves listed-out records unedited */
int tr_list_dirbits(const uint64_t *d_list, uint32_t nlist, int exclude, uint64_t n, uint8_t *d_bits, void *stream);
int tr_launch_pass(const TrPass *p, void *temp, size_t temp_bytes, void *stream);
#ifdef __cplusplus
}
#endif
#endif
