/*
 * tcpprep.h -- C-ABI of the MI355X-native tcpprep classification pass
 * (libtcpedit_hip.so), SURVEY.md 8(f) rank 2: it writes the v04 cache file
 * that tcprewrite / tcpreplay-edit read with -c (src/common/cache.c:63-140).
 *
 * Replaces the per-packet half of the reference's tcpprep tool:
 *   - tcpprep_init / tcpprep_close   <- tcpprep_init / tcpprep_close (src/tcpprep_api.c:40-110)
 *   - tcpprep_parse_args             <- the AutoOpts option surface tcpprep_post_args reads
 *                                       (src/tcpprep_opts.def: --cidr, --mac, --port, --reverse,
 *                                       --nonip, --comment, --no-arg-comment, --include, --exclude,
 *                                       --auto, --ratio, --minmask, --maxmask, --services)
 *   - tcpprep_set_pkt_base           <- (new) a shard's first global record number
 *   - tcpprep_cache_pcap             <- process_raw_packets + write_cache
 *                                       (src/tcpprep.c:339-587, src/common/cache.c:146-219)
 * Auto modes bridge/client/server/first/router (--auto, --ratio, --minmask, --maxmask) are served; regex is not.
 * Classification runs in the gfx950 kernel tp_classify; there is no CPU path.
 */
#ifndef TCPPREP_HIP_H
#define TCPPREP_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tcpprep_hip_s tcpprep_hip_t;

/* allocate a context with tcpprep_init's defaults (server ports 0-1023); 0 ok, -1 error */
int tcpprep_init(tcpprep_hip_t **ctx);
/* parse long options (argv[0] is an option, not a program name); 0 ok, -1 error (tcpprep_geterr) */
int tcpprep_parse_args(tcpprep_hip_t *ctx, int argc, char **argv);
/* upper bound of the cache file size for a pcap image of `pcap_len` bytes */
size_t tcpprep_cache_bound(tcpprep_hip_t *ctx, size_t pcap_len);
/* classify every record of a pcap image on the GPU and write the cache file
   (header, comment, packed entries) into out; returns its size or -1 */
int64_t tcpprep_cache_pcap(tcpprep_hip_t *ctx, const void *pcap, size_t pcap_len, void *out, size_t out_cap);
/* device-resident timing: stage the image and index once, then run the
   classification kernel `iters` times; mean kernel ms (hipEvents) and entries */
int tcpprep_time(tcpprep_hip_t *ctx, const void *pcap, size_t pcap_len, int iters, double *ms_kernel,
                 uint64_t *entries);
/* multi-GPU shards (per-packet modes): the number of records before this shard, so
   --include/--exclude P: lists see global record numbers; 0 ok, -1 error */
int tcpprep_set_pkt_base(tcpprep_hip_t *ctx, uint64_t pkt_base);
/* the HIP device the context classifies on (hipSetDevice before staging; -1 = the calling
   thread's current device, the default); 0 ok, -1 error */
int tcpprep_set_device(tcpprep_hip_t *ctx, int device);
/* cache entries (2-bit) the last tcpprep_cache_pcap wrote: the records, less MAC
   mode's short ones; a shard merge places the next shard's entries after them */
int64_t tcpprep_last_entries(tcpprep_hip_t *ctx);
const char *tcpprep_geterr(tcpprep_hip_t *ctx);
int tcpprep_close(tcpprep_hip_t **ctx);

#ifdef __cplusplus
}
#endif
#endif
