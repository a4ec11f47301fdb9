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
typedef struct {
    const uint8_t *img;   /* device capture image (records at off[j]) */
    uint8_t *cache;       /* -K: the device copy edited from pass to pass, else NULL */
    const uint64_t *off;  /* record offsets */
    uint64_t n;
    int32_t swapped, nsec;
    int32_t edit;         /* this pass edits (unique_iteration advanced, send_packets.c:477) */
    uint64_t iteration;   /* unique_iteration - 1 */
    uint64_t *size;       /* per record: output bytes (0: edit failed, not sent) */
    uint64_t *pos;        /* per record: output offset within the pass */
    void *patch;          /* uint4 per record: {at_s, src, at_d, dst} */
    uint8_t *out;         /* the pass's output */
} TrPass;
size_t tr_scan_temp_bytes(uint64_t n);
int tr_launch_pass(const TrPass *p, void *temp, size_t temp_bytes, void *stream);
#ifdef __cplusplus
}
#endif
#endif
