/*
 * tcpedit.h -- C-ABI of the MI355X-native libtcpedit (libtcpedit_hip.so).
 *
 * Drop-in for the reference's public tcpedit interface (appneta/tcpreplay
 * 4.5.5, src/tcpedit/tcpedit.h:38-55, parse_args.h, tcpedit_api.h:32-58):
 * the same entry points, argument meaning and return codes
 * (TCPEDIT_ERROR -1, TCPEDIT_SOFT_ERROR -2, TCPEDIT_OK 0, TCPEDIT_WARN 1,
 * tcpedit_types.h:31-34), plus
 *   - an option surface that replaces the AutoOpts globals tcpedit_post_args()
 *     reads (tcpedit_set_option / tcpedit_parse_args), and
 *   - a batch entry point (tcpedit_batch_*) that stages a whole pcap image in
 *     HBM and runs the per-packet edit for every record on the GPU in one pass.
 *
 * Every edit runs in the gfx950 kernels: tcpedit_packet() itself launches the
 * same kernel on a one-record batch.  There is no CPU edit path.
 */
#ifndef TCPEDIT_HIP_H
#define TCPEDIT_HIP_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <sys/time.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TCPEDIT_SOFT_ERROR -2
#define TCPEDIT_ERROR -1
#define TCPEDIT_OK 0
#define TCPEDIT_WARN 1

#ifndef PCAP_ERRBUF_SIZE
/* libpcap's record header (pcap/pcap.h); layout-identical when pcap.h is absent */
struct pcap_pkthdr {
    struct timeval ts;
    uint32_t caplen;
    uint32_t len;
};
#endif

#ifndef TCPR_DIR_T_DEFINED
#define TCPR_DIR_T_DEFINED
/* src/common/cache.h:76-82 */
typedef enum tcpr_dir_e { TCPR_DIR_ERROR = -1, TCPR_DIR_NOSEND = 0, TCPR_DIR_C2S = 1, TCPR_DIR_S2C = 2 } tcpr_dir_t;
#endif

/* tcpedit_types.h:36-47 */
typedef enum { TCPEDIT_FIXLEN_OFF = 0, TCPEDIT_FIXLEN_PAD, TCPEDIT_FIXLEN_TRUNC, TCPEDIT_FIXLEN_DEL } tcpedit_fixlen;
typedef enum {
    TCPEDIT_TTL_MODE_OFF = 0,
    TCPEDIT_TTL_MODE_SET,
    TCPEDIT_TTL_MODE_ADD,
    TCPEDIT_TTL_MODE_SUB
} tcpedit_ttl_mode;
typedef enum { TCPEDIT_EDIT_BOTH = 0, TCPEDIT_EDIT_C2S, TCPEDIT_EDIT_S2C } tcpedit_direction;
typedef enum { BEFORE_PROCESS, AFTER_PROCESS } tcpedit_coder;
/* plugins/dlt_en10mb/en10mb_types.h:41-52 */
typedef enum {
    TCPEDIT_MAC_MASK_SMAC1 = 1,
    TCPEDIT_MAC_MASK_SMAC2 = 2,
    TCPEDIT_MAC_MASK_DMAC1 = 4,
    TCPEDIT_MAC_MASK_DMAC2 = 8
} tcpedit_mac_mask;
typedef enum { TCPEDIT_VLAN_OFF = 0, TCPEDIT_VLAN_DEL, TCPEDIT_VLAN_ADD } tcpedit_vlan;

/* ---- the context ------------------------------------------------------------
 * A tcpedit_t * from tcpedit_init points at a context whose first bytes are laid
 * out exactly as the reference's tcpedit_t (tcpedit_types.h:49-61 runtime,
 * :91-153 the struct), so a reference tool compiled against its own headers and
 * relinked against this library reads the fields it dereferences directly --
 * tcprewrite.c:103 and tcpreplay.c:169 `tcpedit->fuzz_seed / fuzz_factor`,
 * tcpreplay.c:256 `tcpedit->seed` -- with their derived values.  The library keeps
 * these fields in step with its own derived tables after tcpedit_post_args and
 * every setter.  The list pointers (cidrmap1..dstipmap, portmap) are NULL: the
 * maps live in the device tables, and no caller outside libtcpedit reads them.
 * dlt_ctx points at the context's DLT plugin handle (plugins_api.h). */
typedef struct {
    unsigned long long packetnum;   /* COUNTER (defines.h.in:103, ENABLE_64BITS) */
    unsigned long long total_bytes;
    unsigned long long pkts_edited;
    int dlt1;
    int dlt2;
    char errstr[1024];              /* TCPEDIT_ERRSTR_LEN */
    char warnstr[1024];
} tcpedit_runtime_t;

typedef struct tcpeditdlt_s tcpeditdlt_t;

typedef struct tcpedit_ref_s {
    bool validated;
    tcpeditdlt_t *dlt_ctx;
    tcpedit_runtime_t runtime;
    bool skip_broadcast;
    tcpedit_fixlen fixlen;
    tcpedit_direction editdir;
    bool rewrite_ip;
    uint32_t tcp_sequence_enable;
    uint32_t tcp_sequence_adjust;
    bool fixcsum;
    bool efcs;
    tcpedit_ttl_mode ttl_mode;
    uint8_t ttl_value;
    int tos;
    int flowlabel;
    int tclass;
    void *cidrmap1, *cidrmap2;      /* tcpr_cidrmap_t * */
    void *srcipmap, *dstipmap;
    uint32_t seed;
    void *portmap;                  /* tcpedit_portmap_t * */
    int mtu;
    bool mtu_truncate;
    int maxpacket;
    uint32_t fuzz_seed;
    uint32_t fuzz_factor;
    bool fixhdrlen;
} tcpedit_ref_t;

typedef struct tcpedit_s tcpedit_t;   /* begins with a tcpedit_ref_t */

/* ---- reference interface: tcpedit.h:38-55 ---------------------------------- */
int tcpedit_init(tcpedit_t **tcpedit, int dlt);                       /* tcpedit.c:371-403 */
char *tcpedit_geterr(tcpedit_t *tcpedit);                              /* tcpedit.c:440-445 */
char *tcpedit_getwarn(tcpedit_t *tcpedit);                             /* tcpedit.c:482-488 */
int tcpedit_checkerror(tcpedit_t *tcpedit, int rcode, const char *prefix); /* tcpedit.c:516-544 */
int tcpedit_validate(tcpedit_t *tcpedit);                              /* tcpedit.c:424-434 */
/* tcpedit.c:46-366 -- edits *pktdata in place (caller's buffer >= MAXPACKET) */
int tcpedit_packet(tcpedit_t *tcpedit, struct pcap_pkthdr **pkthdr, unsigned char **pktdata, tcpr_dir_t direction);
int tcpedit_close(tcpedit_t **tcpedit);                                /* tcpedit.c:551-622 */
int tcpedit_get_output_dlt(tcpedit_t *tcpedit);                        /* tcpedit.c:408-413 */
const unsigned char *tcpedit_l3data(tcpedit_t *tcpedit, tcpedit_coder code, unsigned char *packet, int pktlen); /* :627 */
int tcpedit_l3proto(tcpedit_t *tcpedit, tcpedit_coder code, const unsigned char *packet, int pktlen); /* :642 */
uint64_t tcpedit_get_total_bytes(tcpedit_t *tcpedit);  /* declared tcpedit.h:54-55, never defined there */
uint64_t tcpedit_get_pkts_edited(tcpedit_t *tcpedit);

/* ---- fuzzing.h:26 ------------------------------------------------------------
 * The reference keeps the fuzz RNG in process-wide statics (fuzzing.c:8-20) that
 * tcprewrite.c:103 / tcpreplay.c:169 seed after tcpedit_post_args.  Here the state
 * lives on the device, one word per context: fuzzing_init re-seeds every context's
 * state (and sets the factor) before its next edit.  A context whose tcpedit_post_args
 * derived a --fuzz-seed is seeded with that value by itself when no fuzzing_init call
 * has been made (this library's own tools never need the call). */
void fuzzing_init(uint32_t fuzz_seed, uint32_t fuzz_factor);

/* ---- parse_args.h: derive the per-run tables from the option surface -----
 * The options come from, in this order:
 *   1. tcpedit_parse_args / tcpedit_set_option, when either was called on the context;
 *   2. otherwise the calling tool's AutoOpts descriptor (tcprewriteOptions,
 *      tcpreplayOptions or tcpbridgeOptions), read field by field as libopts lays it
 *      out (libopts/autoopts/options.h:519-579, 603-680) -- so a reference tool
 *      relinked against this library passes its command line through unchanged;
 *   3. otherwise the values the tcpedit_set_* setters stored.
 * With none of the three it fails (TCPEDIT_ERROR) rather than run with no edits. */
int tcpedit_post_args(tcpedit_t *tcpedit);                             /* parse_args.c:34-254 */

/* ---- option surface (stands in for AutoOpts HAVE_OPT/OPT_ARG, Appendix C) --
 * name: long option name without dashes ("seed", "enet-vlan", ...), value: the
 * argument or NULL for flags.  Stacked options (pnat, portmap, enet-subsmac)
 * accumulate.  Returns 0, or -1 for an unknown/duplicate option. */
int tcpedit_set_option(tcpedit_t *tcpedit, const char *name, const char *value);
/* Parses tcpedit/DLT options in argv (long and short forms); arguments it does
 * not know are left for the caller: their indices are written to unused[] (if
 * non-NULL) and counted in the return value (>= 0), or -1 on a parse error. */
int tcpedit_parse_args(tcpedit_t *tcpedit, int argc, char **argv, int *unused);

/* ---- programmatic setters: tcpedit_api.h:32-58 --------------------------- */
int tcpedit_set_encoder_dltplugin_byid(tcpedit_t *, int);            /* tcpedit_api.c:33-65 */
int tcpedit_set_encoder_dltplugin_byname(tcpedit_t *, const char *); /* tcpedit_api.c:72-104 */
int tcpedit_set_skip_broadcast(tcpedit_t *, bool);
int tcpedit_set_fixlen(tcpedit_t *, tcpedit_fixlen);
int tcpedit_set_fixcsum(tcpedit_t *, bool);
int tcpedit_set_fixhdrlen(tcpedit_t *, bool);
int tcpedit_set_efcs(tcpedit_t *, bool);
int tcpedit_set_ttl_mode(tcpedit_t *, tcpedit_ttl_mode);
int tcpedit_set_ttl_value(tcpedit_t *, uint8_t);
int tcpedit_set_tos(tcpedit_t *, uint8_t);
int tcpedit_set_tclass(tcpedit_t *, uint8_t);
int tcpedit_set_flowlabel(tcpedit_t *, uint32_t);
int tcpedit_set_seed(tcpedit_t *);            /* tcpedit_api.c:210: seed = random() */
int tcpedit_set_mtu(tcpedit_t *, int);
int tcpedit_set_mtu_truncate(tcpedit_t *, bool);
int tcpedit_set_maxpacket(tcpedit_t *, int);
int tcpedit_set_cidrmap_s2c(tcpedit_t *, char *);
int tcpedit_set_cidrmap_c2s(tcpedit_t *, char *);
int tcpedit_set_srcip_map(tcpedit_t *, char *);
int tcpedit_set_dstip_map(tcpedit_t *, char *);
int tcpedit_set_port_map(tcpedit_t *, char *);
/* not in tcpedit_api.h, but a setter the reference's struct is edited for directly
 * (tcp_sequence_enable/adjust, tcpedit_types.h:104-105) */
int tcpedit_set_tcp_sequence(tcpedit_t *, uint32_t);

/* ---- EN10MB plugin setters: plugins/dlt_en10mb/en10mb_api.h:38-42 -------- */
int tcpedit_en10mb_set_mac(tcpedit_t *tcpedit, char *mac, tcpedit_mac_mask mask);
int tcpedit_en10mb_set_vlan_mode(tcpedit_t *tcpedit, tcpedit_vlan vlan);
int tcpedit_en10mb_set_vlan_tag(tcpedit_t *tcpedit, uint16_t tag);
int tcpedit_en10mb_set_vlan_priority(tcpedit_t *tcpedit, uint8_t priority);
int tcpedit_en10mb_set_vlan_cfi(tcpedit_t *tcpedit, uint8_t cfi);

/* ---- DLT plugin API: plugins_api.h:29-78 ----------------------------------
 * The context's plugin handle (tcpedit_ref_t.dlt_ctx).  The per-packet plugin
 * hooks (process/decode/encode/merge) have no caller outside libtcpedit: here the
 * L2 decode and encode are fused into the edit kernel, so they are not exported.
 * The accessors answer from the selected decoder/encoder and the L2 walk of the
 * DLT_EN10MB plugin (get_l2len_protocol, get.c:262-451). */
int tcpedit_dlt_post_args(tcpedit_t *tcpedit);                 /* dlt_plugins.c:168-204 */
tcpeditdlt_t *tcpedit_dlt_init(tcpedit_t *tcpedit, int srcdlt);  /* dlt_plugins.c:111-158 */
int tcpedit_dlt_post_init(tcpeditdlt_t *ctx);                   /* dlt_plugins.c:249-262 */
void tcpedit_dlt_cleanup(tcpeditdlt_t *ctx);                    /* dlt_plugins.c:443-474 */
int tcpedit_dlt_output_dlt(tcpeditdlt_t *ctx);                  /* dlt_plugins.c:268-283 */
int tcpedit_dlt_l2len(tcpeditdlt_t *ctx, int dlt, const unsigned char *packet, const int pktlen); /* :290-314 */
int tcpedit_dlt_proto(tcpeditdlt_t *ctx, int dlt, const unsigned char *packet, const int pktlen); /* :320-334 */
unsigned char *tcpedit_dlt_l3data(tcpeditdlt_t *ctx, int dlt, unsigned char *packet, const int pktlen); /* :340 */
int tcpedit_dlt_src(tcpeditdlt_t *ctx);                         /* dlt_plugins.c:424-428 */
int tcpedit_dlt_dst(tcpeditdlt_t *ctx);                         /* dlt_plugins.c:434-438 */

/* ---- batch entry point: a whole pcap image on the GPU ---------------------
 * tcpedit_batch_open copies `pcap` (a complete classic pcap file image,
 * either byte order, us or ns magic) to HBM, builds the record index and the
 * tiles, and uploads `cache` (a tcpprep cache file image, or NULL) for the
 * per-record direction.  pkt_base = 0-based number of the image's first record
 * in the cache (non-zero for a shard of a larger file).  The output of a run
 * stays in HBM until fetched.  For a shard the image may be a record range with
 * a copied 24-byte file header in front. */
typedef struct tcpedit_batch_s tcpedit_batch_t;

typedef struct {
    uint64_t packets, bytes_in, bytes_out, written, edited, soft_errors, warnings, errors, unsupported;
    uint64_t out_len;         /* bytes of the output pcap image (header + written records) */
    int64_t first_error;      /* 0-based record index of the first TCPEDIT_ERROR, or -1 */
    int64_t first_unsupported;/* 0-based record index of the first unsupported record, or -1 */
    uint32_t n_tiles;
    double kernel_ms;         /* device time of the last run (hipEvent) */
    uint32_t fast_lane;       /* 1: the register-resident fast lane ran (size-preserving config) */
    uint32_t generic_tiles;   /* tiles the generic lane edited (all of them without the fast lane) */
    uint32_t fast_kind;       /* fast-lane kernel: 1 te_fast_tiles (block per tile), 2 te_wave_tiles (wave per tile) */
    uint64_t stale_records;   /* written records whose edit read the reference's stale static buffer
                                 (SURVEY Q8), reproduced by the device replay (`unsupported`: those it
                                 could not reproduce -- the run then fails) */
} tcpedit_batch_result_t;

tcpedit_batch_t *tcpedit_batch_open(tcpedit_t *tcpedit, const void *pcap, size_t len, const void *cache,
                                    size_t cache_len, uint64_t pkt_base);
/* a shard of a capture where it lies (e.g. the caller's mmap of the file): the file's
 * 24-byte header and seg_len bytes of whole records, read in place (no host copy), global
 * record numbers from pkt_base -- the per-rank open of a sharded job (tcprewrite.c:289's
 * loop over one rank's byte range) */
tcpedit_batch_t *tcpedit_batch_open_segment(tcpedit_t *tcpedit, const void *hdr, const void *seg, size_t seg_len,
                                            const void *cache, size_t cache_len, uint64_t pkt_base);
int tcpedit_batch_run(tcpedit_t *tcpedit, tcpedit_batch_t *b);     /* TCPEDIT_OK / TCPEDIT_ERROR */
int tcpedit_batch_result(tcpedit_batch_t *b, tcpedit_batch_result_t *r);
size_t tcpedit_batch_output(tcpedit_batch_t *b, void *dst, size_t cap); /* D2H, returns bytes */
/* D2H of the output records only (no file header): a shard's segment of the job's file */
size_t tcpedit_batch_output_records(tcpedit_batch_t *b, void *dst, size_t cap);
const uint8_t *tcpedit_batch_status(tcpedit_batch_t *b);           /* per-record TE_ST_* bytes */
/* times `iters` back-to-back device runs with hipEvents on the run's stream */
int tcpedit_batch_time(tcpedit_t *tcpedit, tcpedit_batch_t *b, int iters, double *ms_per_run);
/* ... and the mean duration of the edit kernel alone (the fast-lane kernel when it runs),
 * from a hipEvent pair around that kernel in every run */
int tcpedit_batch_time_kernels(tcpedit_t *tcpedit, tcpedit_batch_t *b, int iters, double *ms_per_run,
                               double *ms_kernel);
/* the record index rebuilt on the device from the batch's device image (te_index.hip:
 * chunked speculative record-boundary discovery, checked against the chain, then the
 * wave-lane tile cut), replacing the host walk's: `iters` timed builds after one sizing
 * build, *ms = device ms per build.  0 applied; 1 not served (not a wave-lane config, or
 * a guess missed the chain: the host index stays); TCPEDIT_ERROR on error */
int tcpedit_batch_index_device(tcpedit_t *tcpedit, tcpedit_batch_t *b, int iters, double *ms);
void tcpedit_batch_close(tcpedit_batch_t *b);
/* pcapng input: the batch and rewrite calls take a pcapng image as libpcap's
 * reader delivers it to tcprewrite -- classic records, microseconds, the interfaces' link
 * type (te_pcapng.c).  This is that conversion on its own: a malloc'd classic pcap image in
 * *out (free() it); 0, or -1 for a file libpcap would refuse */
int tcpedit_pcapng_to_pcap(const void *in, size_t len, void **out, size_t *out_len);
/* --fuzz-seed across shards.  The reference draws one tcpr_random() per record that
 * reaches the fuzz step from ONE run-wide state (fuzzing.c:8-20,87; tcpedit.c:250-258),
 * so a shard's stream starts after the draws of every earlier shard.
 * tcpedit_batch_fuzz_reach: records of the batch that reach the fuzz step (0 without
 * --fuzz-seed), counted on the device without editing or moving the state; <0 on error.
 * tcpedit_fuzz_skip: advance the context's state by `draws` tcpr_random() calls, as if
 * that many earlier records had reached the step (replaces fuzzing_init's seed for a
 * shard, fuzzing.c:12-20). */
int64_t tcpedit_batch_fuzz_reach(tcpedit_t *tcpedit, tcpedit_batch_t *b);
int tcpedit_fuzz_skip(tcpedit_t *tcpedit, uint64_t draws);
/* The en10mb encoder's dst_modified across shards (a cooked, Juniper or 802.11
 * decoder into en10mb without --enet-dmac; en10mb.c:597,612-615 set it on C2S records and
 * S2C records keep it, so a shard's first records read what an earlier shard left).
 * tcpedit_batch_l2carry_out: the value the batch's last writer leaves (0 or 1), or 2 when
 * no record of it writes (or the config has no carry); found on the device before any edit.
 * tcpedit_set_l2carry: seed the context with the nearest earlier shard's value. */
int tcpedit_batch_l2carry_out(tcpedit_t *tcpedit, tcpedit_batch_t *b);
int tcpedit_set_l2carry(tcpedit_t *tcpedit, int value);

/* DLT_JUNIPER_ETHER across shards (jnpr_ether.c:269-272: a frame whose extensions are not
 * Ethernet is encoded with the decoder state the last whole inner decode left): the state
 * the batch's last whole decode leaves, TCPEDIT_JNPR_STATE_BYTES into `state` -- 1 when
 * the batch has one, 0 when not (or a config without the carry), found before any edit;
 * and seeding a context with an earlier shard's (NULL: the capture's start; unknown = 1:
 * not known, a frame that needs it then fails loudly).  Exchange these before the Q18
 * carry-out (tcpedit_batch_l2carry_out reads the seeded state). */
#define TCPEDIT_JNPR_STATE_BYTES 48
int tcpedit_batch_jnpr_out(tcpedit_t *tcpedit, tcpedit_batch_t *b, void *state, size_t len);
int tcpedit_set_jnpr_state(tcpedit_t *tcpedit, const void *state, size_t len, int unknown);
/* tcpedit_batch_run with the record discovery fused into the edit (the window mode of the
 * wave lane): no index pass or tiles, each wave finds the records of a byte window of the
 * image and edits them in place, the chain checked across windows after.  Batches it does
 * not carry (size-changing or generic-lane configs, a tcpprep cache, big-endian or
 * nanosecond input, a record it leaves to the generic lane) run tcpedit_batch_run: same
 * output.  _time_fused: K such runs back to back, mean ms a run (TCPEDIT_ERROR when not
 * carried); _fused_fallbacks: fused runs that took the exact path. */
int tcpedit_batch_run_fused(tcpedit_t *tcpedit, tcpedit_batch_t *b);
int tcpedit_batch_time_fused(tcpedit_t *tcpedit, tcpedit_batch_t *b, int iters, double *ms_per_run);
uint64_t tcpedit_batch_fused_fallbacks(tcpedit_batch_t *b);

/* tcpreplay-edit's send loop, batched (send_packets.c:379-640; te_replay.c).  The reference
 * edits each packet just before sending it (:469-474, tcpedit_packet with intf1's direction);
 * here one --loop pass over the capture is one device batch.  With preload (--preload-pcap,
 * -K) the first pass edits the records as read and every later pass edits the cached copy
 * in place (get_next_packet :930-980): edits compound from pass to pass.
 * tcpedit_replay_pass writes the pass's records as sent, in the -w dump's form
 * (sendpacket.c:485-486: the edited header, the timestamp fraction as libpcap's nanosecond
 * read leaves it), and returns TCPEDIT_OK or TCPEDIT_ERROR (a hard error: the records before
 * it are in out, as tcpreplay's errx leaves its output). */
typedef struct tcpedit_replay_s tcpedit_replay_t;
tcpedit_replay_t *tcpedit_replay_open(tcpedit_t *tcpedit, const void *pcap, size_t len, int preload);
size_t tcpedit_replay_bound(tcpedit_t *tcpedit, tcpedit_replay_t *r);
int tcpedit_replay_pass(tcpedit_t *tcpedit, tcpedit_replay_t *r, void *out, size_t cap, size_t *out_len);
void tcpedit_replay_close(tcpedit_replay_t *r);
/* tcpreplay's per-record steps around the edit, before the first pass (tcpreplay_opts.def):
 * --include=LIST / --exclude=LIST (send_packets.c:440-447: a listed-out record is neither
 * edited nor sent), --unique-ip and --unique-ip-loops=N (:477-483: fast_edit_packet after
 * the edit, in the same pass).  TCPEDIT_OK or TCPEDIT_ERROR (tcpedit_geterr). */
int tcpedit_replay_parse_args(tcpedit_t *tcpedit, tcpedit_replay_t *r, int argc, char **argv);
/* records whose --unique-ip edit failed so far (tcpreplay's stats->failed) */
uint64_t tcpedit_replay_failed(tcpedit_replay_t *r);
/* new bytes for a batch's records in place (same file and record headers: the index stands) */
int tcpedit_batch_update_input(tcpedit_t *tcpedit, tcpedit_batch_t *b, const void *img, size_t len);
/* the records just before the batch's first (whole records ending where it starts: the previous
 * shard of a sharded job, the previous chunk of a pipelined run), in the batch's format.
 * tcprewrite edits every record in one never-cleared buffer (tcprewrite.c:267-301), so an edit
 * that reads past its record's bytes sees what earlier records left there; when
 * those bytes come from before the batch, the replay walks back into these records.  They are
 * read only then (after a run lists such a record), so the bytes must stay valid until the
 * batch's next run returns.  len 0 clears them. */
int tcpedit_batch_set_prefix(tcpedit_t *tcpedit, tcpedit_batch_t *b, const void *recs, size_t len);

/* device pointers, for callers that keep the data in HBM (e.g. a sender) */
const void *tcpedit_batch_device_output(tcpedit_batch_t *b);
uint64_t tcpedit_batch_input_bytes(tcpedit_batch_t *b);

/* Convenience: H2D + run + D2H of a whole pcap image.  *out is malloc'd. */
int tcpedit_rewrite_pcap(tcpedit_t *tcpedit, const void *in, size_t in_len, const void *cache, size_t cache_len,
                         void **out, size_t *out_len);

/* Pipelined whole-image rewrite into a caller buffer of out_cap >= tcpedit_output_bound()
 * bytes: the image is cut into chunks of whole records (about chunk_bytes each, 0 = 16 MiB),
 * and chunk k's edit overlaps chunk k+1's H2D and chunk k-1's D2H copy.  The buffers are
 * page-locked for the call.  Same output bytes and return codes as tcpedit_rewrite_pcap. */
int tcpedit_rewrite_pcap_pipelined(tcpedit_t *tcpedit, const void *in, size_t in_len, const void *cache,
                                   size_t cache_len, void *out, size_t out_cap, size_t *out_len, size_t chunk_bytes);
/* pipelined calls of this context whose window mode (records found on the device) missed --
 * a chunk's chain miss, a zero-length record, a record reaching more than 64 KiB past its
 * chunk, a record left to the generic lane -- so the call redid the capture on the exact
 * (device-index) pipeline: same output, about twice the time (TCPEDIT_HIP_PIPE_TRACE names
 * the verdict) */
uint64_t tcpedit_pipeline_fallbacks(tcpedit_t *tcpedit);
/* worst-case output image size of `in` under the context's options (host-only walk) */
size_t tcpedit_output_bound(tcpedit_t *tcpedit, const void *in, size_t in_len);
/* page-locked host buffers (a capture read straight into one needs no per-call locking) */
void *tcpedit_host_alloc(size_t bytes);
void tcpedit_host_free(void *p);

/* Introspection (tests): copy the derived per-run device table (te_dev_cfg_t)
 * and, if portlut != NULL, the 65536-entry port map.  Returns its size or -1. */
int tcpedit_get_dev_cfg(tcpedit_t *tcpedit, void *out, size_t len, uint16_t *portlut);

/* select the HIP device used by contexts this thread initialises from now on */
int tcpedit_set_device(int device);

/* Multi-GPU sharding: cut a pcap image into `n`
 * contiguous runs of whole records balanced by bytes, the way libpcap would
 * walk it (a truncated/oversize record ends the walk; the tail stays in the
 * last shard).  On return off[0..n] are record-boundary byte offsets
 * (off[0] = 24, off[n] = end of the walk) and pkt_base[0..n-1] the global
 * 0-based number of each shard's first record, which a shard passes to
 * tcpedit_batch_open so tcpprep cache lookups stay global.  Host-only (no
 * device calls).  Returns the total record count, or -1 on a bad image. */
int64_t tcpedit_pcap_shards(const void *pcap, size_t len, int n, uint64_t *off, uint64_t *pkt_base);

/* Where n shards' outputs go in the job's output file, with tcprewrite's hard-error rule
 * (tcprewrite.c:156-160: the output ends at the first failing record in file order): from
 * each shard's output record bytes (seg_bytes, its records' bytes up to its own first error)
 * and whether it hit a hard error, offset[k] is the file offset of shard k's records and
 * write[k] the bytes it writes (0 for every shard after the first that failed).  Returns
 * the file's size (24 + the bytes written).  Host-only. */
uint64_t tcpedit_shard_place(int n, const uint64_t *seg_bytes, const int *hard_error, uint64_t *offset,
                             uint64_t *write);

#ifdef __cplusplus
}
#endif
#endif
