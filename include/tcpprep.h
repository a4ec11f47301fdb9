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
 *   - tcpprep_auto_table / _merge    <- (new) the auto modes over shards: the first pass's host
 *                                       table (tree.c's RB tree) of each shard, merged across ranks
 * Auto modes bridge/client/server/first/router (--auto, --ratio, --minmask, --maxmask) and
 * --regex (a host-compiled DFA, tp_regex.c) are served.
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
/* --auto over shards (tcpprep.c:480-587, tree.c): the first pass's host table of this
   shard (at its tcpprep_set_pkt_base) as (key, value) pairs -- key: 1 << 63 | IPv4 address,
   or the one IPv6 key (tree_comp, tree.c:618-621); value: server << 32 | client counts, or
   in --auto=first the complement of the earliest sighting (2 x global record index + 0 source
   / 1 destination).  Writes min(count, cap) pairs and returns the count, or -1 (geterr: the
   reference's len_error abort included) */
int64_t tcpprep_auto_table(tcpprep_hip_t *ctx, const void *pcap, size_t pcap_len, uint64_t *keys, uint64_t *vals,
                           size_t cap);
/* the table every shard classifies with: all ranks' pairs, in any order and with repeats;
   merged per key (counts add, first sightings take the earliest).  Required before
   tcpprep_cache_pcap on a shard with a non-zero record base; 0 ok, -1 error */
int tcpprep_auto_merge(tcpprep_hip_t *ctx, const uint64_t *keys, const uint64_t *vals, size_t n);
/* cache entries (2-bit) the last tcpprep_cache_pcap wrote: the records, less MAC
   mode's short ones; a shard merge places the next shard's entries after them */
int64_t tcpprep_last_entries(tcpprep_hip_t *ctx);
const char *tcpprep_geterr(tcpprep_hip_t *ctx);
int tcpprep_close(tcpprep_hip_t **ctx);

#ifdef __cplusplus
}
#endif
#endif
