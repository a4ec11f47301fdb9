/*
 * te_api.c -- the C-ABI of libtcpedit_hip: context lifecycle (tcpedit.c:371-652),
 * the pcap record index / tile builder, and the batch runner that drives the
 * gfx950 kernel.  Host code only; every packet edit happens on the GPU.
 */
#define _GNU_SOURCE
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#include "te_internal.h"
#include "te_index.h"

#define HIPCHK(t, call)                                                                   \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess) {                                                           \
            if (t)                                                                        \
                te_seterr((t), "HIP error %s at %s:%d", hipGetErrorString(e_), __FILE__, __LINE__); \
            goto fail;                                                                    \
        }                                                                                 \
    } while (0)

/* safe_pcap_next's exit (src/common/utils.c:136-156): a record with len > MAX_SNAPLEN or a
   zero len or caplen ends the run; the output keeps the records before it */
#define TE_READER_ERR "safe_pcap_next ERROR: Invalid packet length: packet %lld"

static __thread int g_device = -1; /* per thread: one host thread may drive each device */

int tcpedit_set_device(int device)
{
    g_device = device;
    return hipSetDevice(device) == hipSuccess ? 0 : -1;
}

/* ------------------------------------------------------------------------- */
/* batch: a pcap image resident in HBM                                       */
/* ------------------------------------------------------------------------- */
struct tcpedit_batch_s {
    tcpedit_t *ctx;
    /* host side */
    int swapped, nsec;
    uint32_t linktype;
    uint64_t n_pkts, n_tiles, in_len, out_cap, scratch_bytes;
    uint64_t pkt_base;
    te_tile_t *tiles;
    uint16_t *pkt_rel;
    uint8_t *status;         /* host copy after a run */
    int status_valid;
    int64_t stop_error_pkt;  /* a record the reader refuses (len > MAX_SNAPLEN): hard error */
    int slot_layout;
    int has_trim;            /* some input record has len < caplen: the reader trims it (sizes shift) */
    int grow_off;            /* a run found a record that broke static_grow placement ... */
    uint32_t grow_off_gen;   /* ... under this cfg_gen: place by scan from then on */
    int last_grow;           /* the last launch placed records by static_grow (+4) or static_shrink (-4) */
    int grow_never;          /* pipelined chunk slots: no rerun on a violation, so always scan */
    uint32_t grow_bad;       /* its violation word, read back */
    int mtu_fast;            /* tiles were cut for the wave lane's --mtu-trunc instances */
    int last_mtu;            /* the last launch placed tiles by the --mtu-trunc prediction */
    int fz_fast;             /* tiles were cut for the wave lane's --fuzz-seed instances */
    int wk_small;            /* tiles were cut for the wave lane's TE_FF_SMALL instances */
    int last_fz;             /* the last launch fuzzed on the wave lane (static_fz placement) */
    uint32_t *d_fzlist;      /* static_fz: the reach list, its count, a word a record */
    uint64_t fzlist_cap;     /* (words) */
    long long *d_tcut;       /* the prediction: n_tiles + 1 prefix (te_mtu_cuts), ... */
    long long *d_tcut_raw;   /* ... from per-64-tile sums (scratch) */
    uint64_t tcut_cap;       /* tiles d_tcut holds */
    int tcut_ok;             /* d_tcut is this tile cut's, for tcut_mtu (0 after any re-cut) */
    int32_t tcut_mtu;
    int fast_tiles;          /* tiles were cut for the fast lane ... */
    int fast_kind;           /* ... of this kind (TE_FAST_BLOCK / TE_FAST_WAVE budgets) */
    uint64_t launches;       /* parity selects the fast lane's tile-list count */
    int last_fast;           /* the last launch ran the fast lane ... */
    uint32_t last_listed;    /* ... and left this many tiles to the generic kernel */
    int gen_hint_ok;         /* last_listed came from a run under config generation gen_hint_gen: */
    uint32_t gen_hint_gen;   /* the generic pass after the wave lane then runs on that many blocks, or not at all */
    int last_skipped;        /* the last launch left the generic pass out */
    int last_fgrid;          /* blocks of the last wave-lane launch (slots it wrote) */
    uint64_t *slots_host;    /* their {packets, bytes, edited, -} totals, read back after a run */
    hipEvent_t *kev;         /* event pool for tcpedit_batch_time_kernels (2 per run) */
    int idx_pinned;          /* tiles / pkt_rel are pinned arrays of fixed capacity (a pipeline slot) */
    /* the device index (tcpedit_batch_index_device): the cut walk_range made, and whether
       the device can make it (wave-lane tiles over contiguous records) */
    uint32_t cut_budget, cut_max_pkts, cut_growth;
    uint64_t cut_tiles; /* the walk's greedy tile count (before balance_tiles re-cuts a small batch) */
    int cut_device_ok;
    uint8_t ohdr[24];        /* the output file header, the source of its upload */
    uint8_t *res_pinned;     /* pipeline slot: page-locked landing area of a run's counters, error
                                words and wave-lane slots (a D2H into pageable memory would block) */
    uint64_t idx_cap_tiles, idx_cap_pkts;
    uint8_t *one_img;        /* tcpedit_packet's staging: page-locked record image, then its output */
    /* stale static-buffer reads: the edit's list of records to replay */
    uint8_t *d_q8;           /* q8_cap entries of 16 bytes */
    uint32_t q8_cap;
    int q8_defer;            /* tcpedit_packet replays itself, over the caller's buffer */
    uint8_t *d_q8_init;      /* tcpedit_packet: the caller's buffer bytes [0, need) */
    const uint8_t *pre_host; /* tcpedit_batch_set_prefix: the records before the batch (caller's) */
    size_t pre_len;
    int pre_staged;          /* their last records are on the device: */
    uint8_t *d_pre;          /*   bytes */
    uint64_t *d_pre_off;     /*   offsets of npre records */
    uint32_t npre;
    int pre_file_start;      /*   the first of them is the capture's first record */
    uint64_t walk_from;      /* the walk's first record (0: 24, the image's first) */
    uint64_t rec0;           /* image offset of the launch's first record (0: 24) */
    uint64_t out_base;       /* output offset of its first record in d_out (0: 24; = rec0 mod 16) */
    uint64_t walk_limit;     /* records starting here or later are not the batch's (0: none) */
    uint64_t walk_end;       /* image offset where the record walk stopped ... */
    int walk_stop;           /* ... because: 0 bytes ran out, 1 libpcap's oversize stop, 2 a hard error */
    int kev_n;
    /* the parallel record walk's per-stretch index arrays, kept for the batch's next walk */
    te_tile_t *wk_tiles[64];
    uint16_t *wk_rel[64];
    uint64_t wk_cap_t[64], wk_cap_p[64];
    /* device side */
    uint8_t *d_in, *d_out, *d_status, *d_scratch, *d_dirbits;
    uint64_t dirbits_len;
    te_tile_t *d_tiles;
    uint16_t *d_pkt_rel;
    uint8_t *d_ws;           /* err[0..2] | ticket, done | counters | tile_state[] | list count */
    uint32_t *d_tile_list;   /* fast lane: tiles left to the generic kernel */
    uint32_t last_cnt_off;   /* workspace offset of the last launch's counter set */
    uint64_t *d_l2carry;     /* 2 x (l2carry_cap + 1) scan results, then keys */
    uint64_t l2carry_cap;
    void *d_l2tmp;           /* ... and the scan's scratch */
    size_t l2tmp_bytes;
    uint8_t *d_jnpr;         /* DLT_JUNIPER_ETHER: (jnpr_cap + 1) x {scan, key, 32-byte state} */
    uint64_t jnpr_cap;
    void *d_jtmp;
    size_t jtmp_bytes;
    uint32_t *d_fuzz;        /* --fuzz-seed: per-record RNG states, then a word per 1024 records */
    uint64_t fuzz_cap;       /* records d_fuzz has room for */
    int fuzz_probe_only;     /* the next launch only counts records reaching the fuzz step */
    int q18_only;            /* the next launch only finds the Q18 carry (--fuzz-seed: after the states) */
    uint64_t ws_bytes;
    hipEvent_t ev0, ev1;
    /* window mode (tcpedit_batch_run_fused): its per-window workspace, and the window
       request a launch takes when set */
    uint8_t *d_win;
    uint64_t win_cap;        /* windows d_win has room for */
    const struct te_win_req_s *win_req;
    uint64_t win_fallbacks;  /* fused runs that went the exact way */
    /* results */
    uint64_t counters[TE_CNT__N];
    uint64_t err[3];
    double kernel_ms;
    int ran;
};

#define TE_Q8_CAP (1u << 22) /* stale-read records one batch may list for replay (more fail loudly) */
#define TE_Q8_PRE_RECS 16384u     /* prefix records staged for the replay, at most ... */
#define TE_Q8_PRE_BYTES (32u << 20) /* ... and bytes */
#define TE_Q8_THREADS 256u /* replay threads (scratch: te_q8_slot_bytes() each, per context) */
#define WS_ERR 0
#define WS_ZERO 0
#define WS_TICKET 24
#define WS_GROW_BAD 28   /* u32: a record broke static_grow placement (zeroed with the error words) */
#define WS_COUNTERS 32   /* counter set 0 (TE_CNT__N words) */
#define WS_COUNTERS1 128 /* counter set 1: the fast lane alternates sets by launch parity */
#define WS_STATE 256
#define WS_LIST_CNT(n_tiles) (WS_STATE + 8 * ((n_tiles) + 1))
#define WS_SLOTS(n_tiles) ((WS_LIST_CNT(n_tiles) + 8 + 15) & ~(uint64_t)15) /* wave lane: TE_WK_SLOT_WORDS a block */

/* no edit step can change a record's length or drop it: efcs, VLAN add/del,
 * fixlen, MTU truncation and skipped soft errors are the only ways (plus
 * zero-length records, checked per batch) */
/* libpcap's linktype_to_dlt for the link types this build decodes: LINKTYPE_RAW (101)
 * is DLT_RAW (12); the others are their DLT values */
static uint32_t te_linktype_dlt(uint32_t lt) { return lt == 101 ? 12u : lt; }

static int static_capable(const te_dev_cfg_t *c)
{
    return !c->efcs && c->vlan == TE_VLAN_OFF && c->fixlen == TE_FIXLEN_OFF && !c->mtu_truncate &&
           !c->skip_soft_errors && c->encoder == TE_ENC_EN10MB && c->decoder == TE_DEC_EN10MB && !c->fuzz_seed;
}

/* options the register-resident fast lane carries (fast_lane.hpp): the MAC (with
 * --enet-subsmac and --enet-mac-seed), port,
 * address and seed edits, the IP header edits (TOS, TTL, traffic class, flow label,
 * TCP sequence) and both checksum modes (--fixcsum or incremental); anything else
 * keeps every packet on the generic lane */
/* the CIDR maps fit the config's inline lists (the fast lanes read no spill list) */
static int cidr_inline(const te_dev_cfg_t *c)
{
    return c->n_cidrmap1 <= TE_MAX_CIDRMAP && c->n_cidrmap2 <= TE_MAX_CIDRMAP && c->n_srcipmap <= TE_MAX_CIDRMAP &&
           c->n_dstipmap <= TE_MAX_CIDRMAP;
}

static int fast_capable(const te_dev_cfg_t *c)
{
    return static_capable(c) && !c->fixhdrlen && cidr_inline(c);
}

/* the most one encode can grow a record's L2 header: an encoder header longer than the
   decoded one (a VLAN push is counted by the callers) */
static int l2_growth(const te_dev_cfg_t *c)
{
    const int dl = te_decoder_l2len(c->decoder);
    return c->encoder == TE_ENC_USER                                     ? c->user_length - dl
           : c->encoder == TE_ENC_HDLC                                   ? 4 - dl
           : c->encoder == TE_ENC_EN10MB && c->decoder != TE_DEC_EN10MB
               ? (c->vlan == TE_VLAN_ADD ? 18 : 14) - dl /* another DLT -> Ethernet (en10mb.c:545-549) */
                                                                         : 0;
}
static uint32_t rec_growth(const te_dev_cfg_t *c)
{
    const int l2 = l2_growth(c);
    const uint32_t g = l2 > 4 ? (uint32_t)l2 : 4u;
    return c->fuzz_seed ? 2 * g : g; /* a fuzzed record is encoded twice (tcpedit.c:250-258) */
}

/* the generic lane's slot headroom (te_dev_cfg_t.slot_head): room for the record header to
   move left by every growth the record's encodes can make together -- one encode, or two
   for a fuzzed record, which goes back to `again:` and is decoded (by the input decoder,
   whose L2 is never shorter than te_decoder_l2len) and encoded a second time
   (tcpedit.c:89-118,250-258) */
uint32_t te_slot_head(const te_dev_cfg_t *c)
{
    int g = l2_growth(c);
    if (c->encoder == TE_ENC_EN10MB && c->vlan == TE_VLAN_ADD && g < 4)
        g = 4; /* a VLAN push (en10mb.c:568-578) */
    if (g < 0)
        g = 0;
    const uint32_t need = (uint32_t)(c->fuzz_seed ? 2 * g : g);
    const uint32_t h = (need + 15u) & ~15u;
    return h > TE_HEAD ? h : TE_HEAD;
}

/* VLAN add as the only size change, on the wave lane (static +4 placement): the other
 * fast-lane conditions, and a tag to push (an untagged frame without one is an error) */
static int fast_capable_grow(const te_dev_cfg_t *c)
{
    return c->encoder == TE_ENC_EN10MB && c->decoder == TE_DEC_EN10MB && c->vlan == TE_VLAN_ADD &&
           c->vlan_tag < 65535 && !c->efcs &&
           !c->fuzz_seed && c->fixlen == TE_FIXLEN_OFF && !c->mtu_truncate && !c->skip_soft_errors &&
           !c->fixhdrlen && cidr_inline(c);
}

/* a VLAN pop (--enet-vlan=del) or --efcs as the only size change: every record can shrink
 * by exactly 4 bytes (a record that does not -- untagged, caplen != len, an error -- breaks
 * the static placement and the batch is placed by scan instead).  Returns the TE_SZ_ kind. */
static int static_shrink_kind(const te_dev_cfg_t *c)
{
    if (c->encoder != TE_ENC_EN10MB || c->decoder != TE_DEC_EN10MB || c->vlan == TE_VLAN_ADD ||
        c->fixlen != TE_FIXLEN_OFF || c->mtu_truncate || c->skip_soft_errors || c->fuzz_seed)
        return TE_SZ_NONE;
    if (c->efcs && c->vlan == TE_VLAN_OFF)
        return TE_SZ_EFCS;
    if (!c->efcs && c->vlan == TE_VLAN_DEL)
        return TE_SZ_VDEL;
    return TE_SZ_NONE;
}

/* ... and the wave lane carries it (its fast-lane conditions) */
static int fast_capable_shrink(const te_dev_cfg_t *c)
{
    return static_shrink_kind(c) != TE_SZ_NONE && !c->fixhdrlen && cidr_inline(c);
}

/* --mtu-trunc as the only size change, on the wave lane: records keep their order and
 * lose only their tails, so tile t's output sits at its input offset less the bytes the
 * records before it lose -- a prefix the device predicts from the record headers
 * (te_mtu_cuts) and every tile checks.  (mtu >= 128: a cut packet keeps its whole
 * header window, fast_lane.hpp.) */
static int fast_capable_mtu(const te_dev_cfg_t *c)
{
    return c->encoder == TE_ENC_EN10MB && c->decoder == TE_DEC_EN10MB && c->mtu_truncate &&
           c->mtu >= 128 && c->mtu <= 65535 && c->vlan == TE_VLAN_OFF && !c->efcs && c->fixlen == TE_FIXLEN_OFF &&
           !c->skip_soft_errors && !c->fuzz_seed && !c->fixhdrlen && cidr_inline(c);
}

/* --fuzz-seed on the wave lane: no edit before the fuzz step but the en10mb decode and
 * re-encode (so fuzzing() sees the input bytes and each record's cut is predictable from
 * them, te_fuzz_tile_cut), no other size change, no skipped soft errors (a cut record is a
 * soft error that stays in the output) */
static int fast_capable_fuzz(const te_dev_cfg_t *c)
{
    return c->fuzz_seed && c->encoder == TE_ENC_EN10MB && c->decoder == TE_DEC_EN10MB && c->vlan == TE_VLAN_OFF &&
           !c->efcs && c->fixlen == TE_FIXLEN_OFF && !c->mtu_truncate && !c->skip_soft_errors && !c->fixhdrlen &&
           !c->l2carry && cidr_inline(c) && !(c->mac_mask || c->n_subs || c->random_set) && !c->has_portmap &&
           c->tos < 0 && c->ttl_mode == TE_TTL_OFF && c->tclass < 0 && c->flowlabel < 0 && !c->tcp_sequence_enable;
}

/* TCPEDIT_HIP_NO_FUZZ_FAST=1 keeps --fuzz-seed on the generic lane (A/B checks) */
static int fuzz_fast_off(void)
{
    const char *e = getenv("TCPEDIT_HIP_NO_FUZZ_FAST");
    return e && *e == '1';
}

/* TCPEDIT_HIP_NO_MTU_FAST=1 keeps --mtu-trunc on the generic lane (A/B checks) */
static int mtu_fast_off(void)
{
    const char *e = getenv("TCPEDIT_HIP_NO_MTU_FAST");
    return e && *e == '1';
}

/* IPv6 rewrites with a non-octet target mask keep the reference's stray write
 * (SURVEY Q9): those packets stay on the generic lane */
static int fast_v6_ok(const te_dev_cfg_t *c)
{
    const te_cidrmap_t *lists[4] = {c->cidrmap1, c->cidrmap2, c->srcipmap, c->dstipmap};
    const int n[4] = {c->n_cidrmap1, c->n_cidrmap2, c->n_srcipmap, c->n_dstipmap};
    for (int l = 0; l < 4; l++)
        for (int i = 0; i < n[l] && i < TE_MAX_CIDRMAP; i++) /* (a longer list keeps the generic lane) */
            if (lists[l][i].to.family == 6 && lists[l][i].to.masklen % 8)
                return 0;
    return 1;
}

/* TCPEDIT_HIP_NO_GROW=1 places VLAN-add outputs by scan + look-back (A/B checks) */
static int grow_off_env(void)
{
    const char *e = getenv("TCPEDIT_HIP_NO_GROW");
    return e && *e && strcmp(e, "0") != 0;
}

/* TCPEDIT_HIP_FAST_KIND=block selects te_fast_tiles (one block per tile) for A/B
 * checks; the default is te_wave_tiles (one wave per tile) */
static int fast_kind_pref(void)
{
    const char *e = getenv("TCPEDIT_HIP_FAST_KIND");
    return e && strcmp(e, "block") == 0 ? TE_FAST_BLOCK : TE_FAST_WAVE;
}

static uint32_t rd32(const uint8_t *p, int swapped)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return swapped ? __builtin_bswap32(v) : v;
}

/* One stretch of the record walk (what libpcap's pcap_next does for tcprewrite.c:289):
 * records from `start` on, cut into tiles, until a record would start at or past
 * `stop_at` (the next stretch's first record), the bytes run out, or libpcap stops.
 * Tile first_pkt and scratch_off are relative to the stretch. */
typedef struct {
    /* the cut (same for every stretch).  Offsets are file offsets: record bytes at file
       offset o (o >= 24) are recs[o - 24], so no pointer before the caller's records is
       ever formed (a shard's records may start its buffer) */
    const uint8_t *recs;
    size_t len;
    int swapped, pad, slot_mode, grow_fast, wave, shrink_fast;
    uint32_t budget, max_pkts;
    uint32_t head;           /* slot headroom (te_slot_head) */
    uint32_t growth;         /* output room per record beyond its input (rec_growth) */
    /* the stretch */
    size_t start, stop_at;
    te_tile_t *tiles;
    uint16_t *pkt_rel;
    uint64_t n_tiles, n_pkts, cap_tiles, cap_pkts;
    int fixed;               /* the arrays cannot grow (a pipeline slot's pinned index) */
    uint64_t rec_bytes;      /* sum of 16 + data + 4 (output room) */
    uint64_t scratch_bytes;
    int has_trim;
    int64_t stop_error_pkt;  /* stretch-relative, or -1 */
    int walk_stop;           /* 0 ran out / reached stop_at, 1 oversize, 2 hard error */
    size_t end;              /* offset of the first record not taken */
    int fail;                /* 1 index overflow, 2 out of memory, 3 too many records */
} te_walk_t;

static int walk_grow(void **arr, uint64_t *cap, size_t elem, int fixed)
{
    if (fixed)
        return -1;
    void *n = realloc(*arr, elem * (*cap) * 2);
    if (!n)
        return -1;
    *arr = n;
    *cap *= 2;
    return 0;
}

static void walk_range(te_walk_t *w)
{
    const uint8_t *recs = w->recs;
    const size_t len = w->len;
    size_t off = w->start;
    te_tile_t cur;
    memset(&cur, 0, sizeof(cur));
    uint32_t cur_slots = 0;
    int open = 0;
#define TE_PUSH_TILE()                                                                          \
    do {                                                                                        \
        if (w->n_tiles == w->cap_tiles &&                                                      \
            walk_grow((void **)&w->tiles, &w->cap_tiles, sizeof(te_tile_t), w->fixed) < 0) {    \
            w->fail = w->fixed ? 1 : 2;                                                         \
            goto out;                                                                           \
        }                                                                                       \
        w->tiles[w->n_tiles++] = cur;                                                           \
    } while (0)
    /* the walk is a dependent chain of header loads at record strides the hardware
       prefetcher does not follow (IMIX: ~100 ns a record): stream the lines 4 KiB ahead */
    size_t pf = off;
    while (off + 16 <= len && off < w->stop_at) {
        for (const size_t pf_end = off + 4096 < len ? off + 4096 : len; pf < pf_end; pf += 64)
            __builtin_prefetch(recs + (pf - 24));
        uint32_t caplen = rd32(recs + (off - 24) + 8, w->swapped), plen = rd32(recs + (off - 24) + 12, w->swapped);
        if (caplen > 262144u) { /* libpcap stops at an oversize record ... */
            w->walk_stop = 1;
            break;
        }
        if (off + 16 + caplen > len)
            break; /* ... and at a truncated one (or a pipeline chunk ends here) */
        if (plen > 262144u || plen == 0 || caplen == 0) {
            /* safe_pcap_next (tcprewrite.c:289 -> src/common/utils.c:136-156) exit(-1)s
               here: the output keeps the earlier records */
            w->stop_error_pkt = (int64_t)w->n_pkts;
            w->walk_stop = 2;
            break;
        }
        if (plen < caplen) /* utils.c:159-162: the edit sees caplen = len (sizes shift) */
            w->has_trim = 1;
        uint32_t data = w->pad && plen > caplen ? plen : caplen;
        uint32_t g = (uint32_t)(off & 15);
        uint32_t slot = TE_SLOT_BYTES_OF_H(w->head, g, data);
        int huge, fits;
        if (w->slot_mode && !w->grow_fast) {
            huge = slot > TE_SLOT_BYTES;
            fits = open && cur_slots + slot <= TE_SLOT_BYTES;
        } else {
            huge = !TE_CONTIG_FITS_IN(g, 16 + caplen, w->budget);
            fits = open && TE_CONTIG_FITS_IN(cur.span_off & 15, off + 16 + caplen - cur.span_off, w->budget);
        }
        /* wave lane: a record too large for a wave image but not for the generic kernel's
           LDS slot is a tile of its own, left to the generic kernel (no HBM scratch) */
        const int solo =
            huge && w->wave && (w->slot_mode ? slot <= TE_SLOT_BYTES : TE_CONTIG_FITS(g, 16 + caplen));
        if (solo)
            huge = 0;
        if (open && (huge || solo || cur.npkt >= w->max_pkts || !fits)) {
            TE_PUSH_TILE();
            open = 0;
        }
        if (!open) {
            memset(&cur, 0, sizeof(cur));
            cur.span_off = off;
            cur.first_pkt = (uint32_t)w->n_pkts;
            cur.scratch_off = TE_NO_SCRATCH;
            cur_slots = 0;
            open = 1;
        }
        if (w->n_pkts == w->cap_pkts &&
            walk_grow((void **)&w->pkt_rel, &w->cap_pkts, sizeof(uint16_t), w->fixed) < 0) {
            w->fail = w->fixed ? 1 : 2;
            goto out;
        }
        w->pkt_rel[w->n_pkts++] = (uint16_t)(off - cur.span_off);
        cur.npkt++;
        cur.span_len = (uint32_t)(off + 16 + caplen - cur.span_off);
        cur_slots += slot;
        w->rec_bytes += 16 + (uint64_t)data + w->growth;
        if (huge) { /* a record larger than a tile: its slot lives in HBM scratch */
            cur.scratch_off = w->scratch_bytes;
            w->scratch_bytes += (slot + TE_LDS_FRONT + 64 + 255) & ~255u;
            TE_PUSH_TILE();
            open = 0;
        } else if (solo) {
            cur.flags |= TE_TILE_SOLO;
            TE_PUSH_TILE();
            open = 0;
        }
        off += 16 + caplen;
        if (w->n_pkts >= 0xffffffffull) {
            w->fail = 3;
            goto out;
        }
    }
    if (open)
        TE_PUSH_TILE();
out:
#undef TE_PUSH_TILE
    w->end = off;
}

/* Tile balance for small batches.  Wave w of the wave lane's W takes tiles w, w + W, ...
 * (static dealing), so a batch of T tiles runs ceil(T / W) rounds and, when T is just
 * past a multiple of W, its last round has few waves busy: latency-bound, nearly as long
 * as a full one (C2: 15,873 greedy tiles of 63 records over 5,120 waves is 3.1 rounds,
 * timed as 4).  Re-cut the record sequence to ceil(n / (R W)) records a tile, R = the
 * rounds the greedy cut needs, so every wave takes R tiles of the same size.  Tiles of
 * one record too large for the image (solo, scratch) stay as they are and bound the
 * re-cut; every new tile satisfies the walk's budget test.  Only for batches of a few
 * rounds (the tail is 1/R of the run) whose tiles are count- rather than byte-limited. */
#define TE_BALANCE_MAX_ROUNDS 8
static int balance_tiles(tcpedit_batch_t *b, uint32_t waves, uint32_t budget, uint32_t max_pkts)
{
    const uint64_t T = b->n_tiles, n = b->n_pkts;
    const char *e = getenv("TCPEDIT_HIP_BALANCE");
    if ((e && *e == '0') || !waves || T == 0 || T > (uint64_t)waves * TE_BALANCE_MAX_ROUNDS)
        return 0;
    const uint64_t R = (T + waves - 1) / waves, target = R * waves;
    const uint64_t per = (n + target - 1) / target;
    if (per >= max_pkts || T * 100 >= target * 97) /* byte-limited tiles, or balanced already */
        return 0;
    te_tile_t *nt = malloc(sizeof(te_tile_t) * (target + T + 16));
    if (!nt)
        return 0; /* the greedy cut stands */
    uint64_t cnt = 0;
    te_tile_t cur;
    int open = 0;
    for (uint64_t t = 0; t < T; t++) {
        const te_tile_t ot = b->tiles[t];
        if ((ot.flags & TE_TILE_SOLO) || ot.scratch_off != TE_NO_SCRATCH) {
            if (open)
                nt[cnt++] = cur, open = 0;
            nt[cnt++] = ot;
            continue;
        }
        const uint64_t tend = ot.span_off + ot.span_len;
        for (uint32_t k = 0; k < ot.npkt; k++) {
            const uint32_t j = ot.first_pkt + k;
            const uint64_t off = ot.span_off + b->pkt_rel[j];
            const uint64_t end = k + 1 < ot.npkt ? ot.span_off + b->pkt_rel[j + 1] : tend;
            if (open && (cur.npkt >= per || !TE_CONTIG_FITS_IN(cur.span_off & 15, end - cur.span_off, budget)))
                nt[cnt++] = cur, open = 0;
            if (!open) {
                memset(&cur, 0, sizeof(cur));
                cur.span_off = off;
                cur.first_pkt = j;
                cur.scratch_off = TE_NO_SCRATCH;
                open = 1;
            }
            /* (record j's old offset was read above, before this write) */
            b->pkt_rel[j] = (uint16_t)(off - cur.span_off);
            cur.npkt++;
            cur.span_len = (uint32_t)(end - cur.span_off);
        }
    }
    if (open)
        nt[cnt++] = cur;
    free(b->tiles);
    b->tiles = nt;
    b->n_tiles = cnt;
    return 1;
}

/* a plausible record chain at p: `n` consecutive headers within the image whose
   lengths libpcap would accept and whose microsecond/nanosecond field is in range */
static int chain_plausible(const uint8_t *recs, size_t len, size_t p, int swapped, int nsec, int n)
{
    for (int i = 0; i < n; i++) {
        if (p + 16 > len)
            return i > 0;
        const uint8_t *h = recs + (p - 24); /* (file offset p >= 24) */
        const uint32_t frac = rd32(h + 4, swapped), cl = rd32(h + 8, swapped), pl = rd32(h + 12, swapped);
        if (cl > 262144u || pl > 262144u || frac >= (nsec ? 1000000000u : 1000000u) || p + 16 + cl > len)
            return 0;
        p += 16 + cl;
    }
    return 1;
}

static int walk_threads(void)
{
    static int n = 0;
    if (!n) {
        const char *e = getenv("TCPEDIT_HIP_WALK_THREADS");
        n = e && atoi(e) > 0 ? atoi(e) : 8;
        if (n > 64)
            n = 64;
    }
    return n;
}

/* A small process-wide pool of walker threads (created on first use; thread creation
 * per chunk cost about as much as the walk itself).  Jobs carry their caller's
 * pending counter, so concurrent callers share the pool safely.  A forked child
 * starts without the threads, so it starts a pool of its own. */
typedef struct {
    te_walk_t *w;
    int *pending;
} te_job_t;
#define TE_POOL_Q 256
static pthread_mutex_t pool_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t pool_cv = PTHREAD_COND_INITIALIZER, pool_done = PTHREAD_COND_INITIALIZER;
static te_job_t pool_q[TE_POOL_Q];
static int pool_head, pool_tail, pool_n, pool_atfork;

static void pool_child_reset(void)
{
    pthread_mutex_init(&pool_mu, NULL);
    pthread_cond_init(&pool_cv, NULL);
    pthread_cond_init(&pool_done, NULL);
    pool_head = pool_tail = pool_n = 0;
}

static void *pool_worker(void *arg)
{
    (void)arg;
    for (;;) {
        pthread_mutex_lock(&pool_mu);
        while (pool_head == pool_tail)
            pthread_cond_wait(&pool_cv, &pool_mu);
        te_job_t j = pool_q[pool_head % TE_POOL_Q];
        pool_head++;
        pthread_mutex_unlock(&pool_mu);
        walk_range(j.w);
        pthread_mutex_lock(&pool_mu);
        (*j.pending)--;
        pthread_cond_broadcast(&pool_done);
        pthread_mutex_unlock(&pool_mu);
    }
    return NULL;
}

/* queue a stretch; returns 0, or -1 (the caller then walks it itself) */
static int pool_submit(te_walk_t *w, int *pending, int want_threads)
{
    pthread_mutex_lock(&pool_mu);
    if (!pool_atfork) {
        pthread_atfork(NULL, NULL, pool_child_reset);
        pool_atfork = 1;
    }
    while (pool_n < want_threads) {
        pthread_t th;
        if (pthread_create(&th, NULL, pool_worker, NULL) != 0)
            break;
        pthread_detach(th);
        pool_n++;
    }
    if (pool_n == 0 || pool_tail - pool_head >= TE_POOL_Q) {
        pthread_mutex_unlock(&pool_mu);
        return -1;
    }
    pool_q[pool_tail % TE_POOL_Q] = (te_job_t){w, pending};
    pool_tail++;
    (*pending)++;
    pthread_cond_signal(&pool_cv);
    pthread_mutex_unlock(&pool_mu);
    return 0;
}

static void pool_wait(int *pending)
{
    pthread_mutex_lock(&pool_mu);
    while (*pending)
        pthread_cond_wait(&pool_done, &pool_mu);
    pthread_mutex_unlock(&pool_mu);
}

#define TE_WALK_PART_MIN ((size_t)2 << 20) /* bytes per stretch of a parallel walk, at least */

/* a capture of small records: its first (up to) 256 records average at most
   TE_SMALL_REC_BYTES with their headers, so 64 of them -- the wave tile's record cap -- fill
   the 5 KiB tiles of the TE_FF_SMALL instances (C2's 80-byte records: 63), which run a block
   more per CU than the 8 KiB ones -- for a batch the Infinity Cache holds (in + out <= 256
   MiB): from HBM the 8 KiB tiles' bytes in flight count for more (c2x10 0.645 vs 0.636 of
   peak, C2 0.623 vs 0.679; TCPEDIT_HIP_NO_SMALL=1: never, for A/B) */
#define TE_SMALL_REC_BYTES 84u
#define TE_SMALL_MAX_BATCH ((uint64_t)128 << 20)
static int small_records(const uint8_t *recs, size_t len, int sw)
{
    static int off_env = -1;
    if (off_env < 0) {
        const char *e = getenv("TCPEDIT_HIP_NO_SMALL");
        off_env = e && *e && *e != '0';
    }
    uint64_t off = 0, n = 0;
    while (recs && !off_env && n < 256 && off + 16 <= len) {
        const uint32_t cl = rd32(recs + off + 8, sw);
        if (cl > 262144u || off + 16 + cl > len)
            break;
        off += 16 + cl;
        n++;
    }
    return n >= 16 && off <= n * TE_SMALL_REC_BYTES;
}

/* The tile cut a config and capture (b->swapped, b->nsec; its records recs[0, len) for the
 * small-record test) get: the lane (wave, block or generic), the slot layout, the tile
 * budget; *proto is the walk's prototype. */
static void cut_setup(tcpedit_t *t, tcpedit_batch_t *b, te_walk_t *proto, const uint8_t *recs, size_t len,
                      uint64_t batch_bytes)
{
    memset(proto, 0, sizeof(*proto));
    proto->swapped = b->swapped;
    proto->pad = t->cfg.fixlen == TE_FIXLEN_PAD;
    /* slots with headroom: VLAN push, fixlen pad, a user L2 header longer than Ethernet's */
    proto->slot_mode = proto->pad || (t->cfg.encoder == TE_ENC_EN10MB && t->cfg.vlan == TE_VLAN_ADD) ||
                       l2_growth(&t->cfg) > 0;
    proto->head = te_slot_head(&t->cfg);
    b->slot_layout = proto->slot_mode;
    /* the wave lane also takes VLAN add (native-order microsecond input only): its tiles
       are cut to the wave image (their per-record slots then fit the generic kernel's) */
    proto->grow_fast = !proto->pad && fast_capable_grow(&t->cfg) && !b->swapped && !b->nsec &&
                       fast_kind_pref() == TE_FAST_WAVE;
    /* ... and a VLAN pop or --efcs (native-order microsecond input only) */
    const int shrink_fast = !proto->slot_mode && fast_capable_shrink(&t->cfg) && !b->swapped && !b->nsec;
    /* ... and --mtu-trunc (native-order microsecond input, the wave lane only) */
    b->mtu_fast = !proto->slot_mode && fast_capable_mtu(&t->cfg) && !b->swapped && !b->nsec &&
                  fast_kind_pref() == TE_FAST_WAVE && !mtu_fast_off();
    /* ... and --fuzz-seed (native-order microsecond input, the wave lane only) */
    b->fz_fast = !proto->slot_mode && fast_capable_fuzz(&t->cfg) && !b->swapped && !b->nsec &&
                 fast_kind_pref() == TE_FAST_WAVE && !fuzz_fast_off();
    b->fast_tiles = (!proto->slot_mode && fast_capable(&t->cfg)) || proto->grow_fast || shrink_fast || b->mtu_fast ||
                    b->fz_fast;
    b->fast_kind = b->fast_tiles ? fast_kind_pref() : 0;
    if (shrink_fast && !proto->grow_fast && b->fast_kind != TE_FAST_WAVE) /* (the block lane has no shrink) */
        b->fast_tiles = 0, b->fast_kind = 0;
    proto->wave = b->fast_kind == TE_FAST_WAVE;
    b->wk_small = proto->wave && !proto->grow_fast && !shrink_fast && !b->mtu_fast && !b->fz_fast &&
                  batch_bytes <= TE_SMALL_MAX_BATCH && small_records(recs, len, b->swapped);
    proto->budget = proto->wave      ? te_wave_tile_bytes(&t->cfg, proto->grow_fast ? TE_SZ_GROW
                                                                   : shrink_fast     ? static_shrink_kind(&t->cfg)
                                                                   : b->mtu_fast     ? TE_SZ_MTU
                                                                   : b->fz_fast      ? TE_SZ_FUZZ
                                                                                     : TE_SZ_NONE, b->wk_small)
                    : b->fast_tiles ? TE_FK_TILE_BYTES
                                    : TE_SLOT_BYTES;
    proto->max_pkts = proto->wave ? TE_WK_PKTS : b->fast_tiles ? TE_FK_BLOCK : TE_MAX_PKTS;
    proto->stop_error_pkt = -1;
    proto->growth = rec_growth(&t->cfg);
    proto->shrink_fast = shrink_fast;
    b->cut_budget = proto->budget;
    b->cut_max_pkts = proto->max_pkts;
    b->cut_growth = proto->growth;
    b->cut_device_ok = proto->wave && !proto->pad && (!proto->slot_mode || proto->grow_fast) &&
                       proto->head == TE_HEAD; /* (te_index sizes scratch slots with TE_HEAD) */
}

/* Walk the records and cut them into tiles.  A large image is walked as up to
 * TCPEDIT_HIP_WALK_THREADS stretches at once: stretch i > 0 starts at a guessed record
 * boundary (the first plausible chain of headers after an even split point), and it
 * counts only if stretch i - 1, walking from a known boundary, ends exactly there.
 * From the first stretch that does not, the walk goes on sequentially, so the index is
 * the sequential walk's records whatever the guesses (the tile cut may differ: any cut
 * is valid). */
static int index_image(tcpedit_t *t, tcpedit_batch_t *b, const uint8_t *hdr, const uint8_t *recs, size_t len)
{
    if (len < 24) {
        te_seterr(t, "pcap image too short");
        return -1;
    }
    uint32_t magic;
    memcpy(&magic, hdr, 4);
    switch (magic) {
    case 0xa1b2c3d4u: b->swapped = 0; b->nsec = 0; break;
    case 0xd4c3b2a1u: b->swapped = 1; b->nsec = 0; break;
    case 0xa1b23c4du: b->swapped = 0; b->nsec = 1; break;
    case 0x4d3cb2a1u: b->swapped = 1; b->nsec = 1; break;
    default:
        te_seterr(t, "not a pcap file (magic 0x%08x)", magic);
        return -1;
    }
    b->linktype = te_linktype_dlt(rd32(hdr + 20, b->swapped) & 0x03ffffffu);
    te_walk_t proto;
    cut_setup(t, b, &proto, recs, len > 24 ? len - 24 : 0, len);
    proto.recs = recs;
    proto.len = len;

    uint64_t cap_tiles = 1024, cap_pk = 1 << 16;
    if (b->idx_pinned) { /* a pipeline slot: the chunk budget bounds both (16 B per record at least) */
        cap_tiles = b->idx_cap_tiles;
        cap_pk = b->idx_cap_pkts;
    } else {
        free(b->tiles);
        free(b->pkt_rel);
        b->tiles = malloc(sizeof(te_tile_t) * cap_tiles);
        b->pkt_rel = malloc(sizeof(uint16_t) * cap_pk);
        if (!b->tiles || !b->pkt_rel) {
            te_seterr(t, "out of host memory");
            return -1;
        }
    }
    /* the stretches: [from, q1), [q1, q2), ..., up to the walk limit (a pipeline chunk's
       records are the ones starting in its own bytes) */
    const size_t from = b->walk_from ? b->walk_from : 24, limit = b->walk_limit ? b->walk_limit : (size_t)-1;
    int parts = walk_threads();
    if ((size_t)parts > (len - 24) / TE_WALK_PART_MIN)
        parts = (int)((len - 24) / TE_WALK_PART_MIN);
    if (parts < 1)
        parts = 1;
    size_t q[65];
    q[0] = from;
    int np = 1;
    for (int i = 1; i < parts; i++) {
        const size_t s0 = from + (len - from) / parts * i, lim = s0 + (1u << 20) < len ? s0 + (1u << 20) : len;
        if (s0 >= limit)
            break;
        size_t p = s0 > q[np - 1] ? s0 : q[np - 1] + 1;
        for (; p + 16 <= lim; p++)
            if (chain_plausible(recs, len, p, b->swapped, b->nsec, 8))
                break;
        if (p + 16 <= lim)
            q[np++] = p;
    }
    q[np] = limit;
    te_walk_t w[64];
    int pending = 0;
    for (int i = 0; i < np; i++) {
        w[i] = proto;
        w[i].start = q[i];
        w[i].stop_at = q[i + 1];
        if (i == 0) { /* stretch 0 writes the batch's own arrays */
            w[i].tiles = b->tiles;
            w[i].pkt_rel = b->pkt_rel;
            w[i].cap_tiles = cap_tiles;
            w[i].cap_pkts = cap_pk;
            w[i].fixed = b->idx_pinned;
        } else { /* the batch's kept arrays for this stretch, grown as the walk needs */
            const uint64_t span = (i + 1 < np ? q[i + 1] : len) - q[i];
            const uint64_t want_p = span / 64 + 64, want_t = span / 1024 + 64;
            if (b->wk_cap_p[i] < want_p) {
                free(b->wk_rel[i]);
                b->wk_rel[i] = malloc(sizeof(uint16_t) * want_p);
                b->wk_cap_p[i] = b->wk_rel[i] ? want_p : 0;
            }
            if (b->wk_cap_t[i] < want_t) {
                free(b->wk_tiles[i]);
                b->wk_tiles[i] = malloc(sizeof(te_tile_t) * want_t);
                b->wk_cap_t[i] = b->wk_tiles[i] ? want_t : 0;
            }
            w[i].tiles = b->wk_tiles[i];
            w[i].pkt_rel = b->wk_rel[i];
            w[i].cap_tiles = b->wk_cap_t[i];
            w[i].cap_pkts = b->wk_cap_p[i];
            if (!w[i].tiles || !w[i].pkt_rel) {
                w[i].fail = 2;
                continue;
            }
            if (pool_submit(&w[i], &pending, walk_threads() - 1) < 0)
                walk_range(&w[i]);
        }
    }
    walk_range(&w[0]);
    pool_wait(&pending);
    /* stitch: stretch i counts while every earlier one ended exactly at its start */
    te_walk_t *m = &w[0];
    int rc = 0, i = 1;
    for (; i < np && !m->fail; i++) {
        te_walk_t *x = &w[i];
        if (m->end != x->start || m->walk_stop || x->fail)
            break;
        if (m->n_tiles + x->n_tiles > m->cap_tiles || m->n_pkts + x->n_pkts > m->cap_pkts) {
            if (m->fixed || walk_grow((void **)&m->tiles, &m->cap_tiles, sizeof(te_tile_t), 0) < 0 ||
                walk_grow((void **)&m->pkt_rel, &m->cap_pkts, sizeof(uint16_t), 0) < 0) {
                m->fail = m->fixed ? 1 : 2;
                break;
            }
            i--; /* grown by 2x: retry this stretch */
            continue;
        }
        for (uint64_t k = 0; k < x->n_tiles; k++) {
            te_tile_t tl = x->tiles[k];
            tl.first_pkt += (uint32_t)m->n_pkts;
            if (tl.scratch_off != TE_NO_SCRATCH)
                tl.scratch_off += m->scratch_bytes;
            m->tiles[m->n_tiles++] = tl;
        }
        memcpy(m->pkt_rel + m->n_pkts, x->pkt_rel, sizeof(uint16_t) * x->n_pkts);
        if (x->stop_error_pkt >= 0)
            m->stop_error_pkt = (int64_t)m->n_pkts + x->stop_error_pkt;
        m->n_pkts += x->n_pkts;
        m->rec_bytes += x->rec_bytes;
        m->scratch_bytes += x->scratch_bytes;
        m->has_trim |= x->has_trim;
        m->walk_stop = x->walk_stop;
        m->end = x->end;
        m->stop_at = x->stop_at;
    }
    if (!m->fail && i < np && !m->walk_stop && m->end + 16 <= len && m->end < limit) {
        /* a guess was wrong (or a stretch failed): the rest, sequentially */
        m->stop_at = limit;
        const size_t from = m->end;
        te_walk_t rest = proto;
        rest.start = from;
        rest.stop_at = limit;
        rest.tiles = m->tiles + m->n_tiles;
        rest.pkt_rel = m->pkt_rel + m->n_pkts;
        rest.cap_tiles = m->cap_tiles - m->n_tiles;
        rest.cap_pkts = m->cap_pkts - m->n_pkts;
        rest.fixed = 1;
        walk_range(&rest);
        if (rest.fail == 1 && !m->fixed) { /* room for the rest: grow to the worst case, walk again */
            const uint64_t need = m->n_pkts + (len - from) / 16 + 2;
            te_tile_t *nt = realloc(m->tiles, sizeof(te_tile_t) * need);
            uint16_t *np2 = nt ? realloc(m->pkt_rel, sizeof(uint16_t) * need) : NULL;
            if (nt)
                m->tiles = nt;
            if (np2)
                m->pkt_rel = np2;
            if (nt && np2) {
                m->cap_tiles = m->cap_pkts = need;
                rest = proto;
                rest.start = from;
                rest.stop_at = limit;
                rest.tiles = m->tiles + m->n_tiles;
                rest.pkt_rel = m->pkt_rel + m->n_pkts;
                rest.cap_tiles = rest.cap_pkts = need - m->n_pkts;
                rest.fixed = 1;
                walk_range(&rest);
            } else {
                rest.fail = 2;
            }
        }
        for (uint64_t k = 0; k < rest.n_tiles; k++) {
            rest.tiles[k].first_pkt += (uint32_t)m->n_pkts;
            if (rest.tiles[k].scratch_off != TE_NO_SCRATCH)
                rest.tiles[k].scratch_off += m->scratch_bytes;
        }
        if (rest.stop_error_pkt >= 0)
            m->stop_error_pkt = (int64_t)m->n_pkts + rest.stop_error_pkt;
        m->n_tiles += rest.n_tiles;
        m->n_pkts += rest.n_pkts;
        m->rec_bytes += rest.rec_bytes;
        m->scratch_bytes += rest.scratch_bytes;
        m->has_trim |= rest.has_trim;
        m->walk_stop = rest.walk_stop;
        m->end = rest.end;
        m->fail = rest.fail;
    }
    for (int j = 1; j < np; j++) { /* keep what the walks grew to */
        if (w[j].tiles) {
            b->wk_tiles[j] = w[j].tiles;
            b->wk_cap_t[j] = w[j].cap_tiles;
        }
        if (w[j].pkt_rel) {
            b->wk_rel[j] = w[j].pkt_rel;
            b->wk_cap_p[j] = w[j].cap_pkts;
        }
    }
    b->tiles = m->tiles;
    b->pkt_rel = m->pkt_rel;
    if (m->fail) {
        te_seterr(t, m->fail == 1 ? "pipeline slot index overflow"
                     : m->fail == 3 ? "too many records for one batch" : "out of host memory");
        rc = -1;
    }
    b->n_tiles = m->n_tiles;
    b->cut_tiles = m->n_tiles;
    b->n_pkts = m->n_pkts;
    if (!rc && proto.wave && !proto.slot_mode && !b->idx_pinned)
        balance_tiles(b, te_wave_waves(&t->cfg, proto.shrink_fast ? static_shrink_kind(&t->cfg)
                                                : b->mtu_fast      ? TE_SZ_MTU
                                                : b->fz_fast       ? TE_SZ_FUZZ
                                                                   : TE_SZ_NONE, b->wk_small),
                      proto.budget, proto.max_pkts);
    b->out_cap = 24 + 64 + m->rec_bytes;
    b->scratch_bytes = m->scratch_bytes;
    b->stop_error_pkt = m->stop_error_pkt;
    b->has_trim = m->has_trim;
    b->walk_stop = m->walk_stop;
    b->walk_end = m->end;
    b->in_len = len;
    return rc;
}

static void batch_free_dev(tcpedit_batch_t *b)
{
    hipFree(b->d_in);
    hipFree(b->d_out);
    hipFree(b->d_status);
    hipFree(b->d_scratch);
    hipFree(b->d_dirbits);
    hipFree(b->d_win);
    hipFree(b->d_tiles);
    hipFree(b->d_pkt_rel);
    hipFree(b->d_ws);
    hipFree(b->d_tcut);
    hipFree(b->d_tcut_raw);
    b->d_tcut = NULL;
    b->d_tcut_raw = NULL;
    b->tcut_cap = 0;
    b->tcut_ok = 0;
    hipFree(b->d_tile_list);
    hipFree(b->d_fuzz);
    hipFree(b->d_fzlist);
    b->d_fzlist = NULL;
    b->fzlist_cap = 0;
    hipFree(b->d_l2carry);
    hipFree(b->d_jnpr);
    hipFree(b->d_jtmp);
    hipFree(b->d_l2tmp);
    b->d_l2carry = NULL;
    b->d_l2tmp = NULL;
    b->l2carry_cap = 0;
    b->l2tmp_bytes = 0;
    hipFree(b->d_q8);
    hipFree(b->d_q8_init);
    b->d_q8 = b->d_q8_init = NULL;
    hipFree(b->d_pre);
    hipFree(b->d_pre_off);
    b->d_pre = NULL;
    b->d_pre_off = NULL;
    b->npre = 0;
    b->pre_staged = 0;
    b->d_fuzz = NULL;
    b->fuzz_cap = 0;
    b->d_tile_list = NULL;
    b->d_in = b->d_out = b->d_status = b->d_scratch = b->d_dirbits = b->d_ws = NULL;
    b->d_tiles = NULL;
    b->d_pkt_rel = NULL;
}

void tcpedit_batch_close(tcpedit_batch_t *b)
{
    if (!b)
        return;
    batch_free_dev(b);
    if (b->ev0)
        hipEventDestroy(b->ev0);
    if (b->ev1)
        hipEventDestroy(b->ev1);
    for (int i = 0; i < b->kev_n; i++)
        hipEventDestroy(b->kev[i]);
    free(b->kev);
    free(b->slots_host);
    for (int i = 0; i < 64; i++) {
        free(b->wk_tiles[i]);
        free(b->wk_rel[i]);
    }
    if (b->res_pinned)
        hipHostFree(b->res_pinned);
    if (b->one_img)
        hipHostFree(b->one_img);
    if (b->idx_pinned) {
        hipHostFree(b->tiles);
        hipHostFree(b->pkt_rel);
    } else {
        free(b->tiles);
        free(b->pkt_rel);
    }
    free(b->status);
    free(b);
}

/* tcpprep cache file image -> its data bytes (cache.c:63-140) */
static int cache_data(tcpedit_t *t, const uint8_t *c, size_t n, const uint8_t **data, uint64_t *dlen)
{
    if (n < 24 || memcmp(c, "tcpprep\0", 8) != 0) {
        te_seterr(t, "not a tcpprep cache file");
        return -1;
    }
    if (strtol((const char *)c + 8, NULL, 10) != 4) {
        te_seterr(t, "cache file version mismatch");
        return -1;
    }
    uint64_t np = 0;
    for (int i = 0; i < 8; i++)
        np = (np << 8) | c[12 + i];
    uint32_t ppb = ((uint32_t)c[20] << 8) | c[21], clen = ((uint32_t)c[22] << 8) | c[23];
    if (ppb == 0) {
        te_seterr(t, "invalid cache header");
        return -1;
    }
    uint64_t sz = np / ppb + (np % ppb ? 1 : 0);
    if (24 + (uint64_t)clen + sz > n) {
        te_seterr(t, "Cache data length doesn't match cache header");
        return -1;
    }
    *data = c + 24 + clen;
    *dlen = sz;
    return 0;
}

/* first device use of a context: pick the device and create its stream */
static int te_dev_ready(tcpedit_t *t)
{
    if (t->stream)
        return 0;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        te_seterr(t, "no HIP device available: libtcpedit_hip edits packets on the GPU only");
        return -1;
    }
    if (t->device >= 0 && hipSetDevice(t->device) != hipSuccess) {
        te_seterr(t, "hipSetDevice(%d) failed", t->device);
        return -1;
    }
    if (hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking) != hipSuccess) {
        te_seterr(t, "hipStreamCreate failed");
        return -1;
    }
    return 0;
}

int te_upload_cfg(tcpedit_t *t)
{
    if (te_dev_ready(t) < 0)
        return -1;
    if (t->cfg.fuzz_seed && te_fuzz_init_gen && t->cfg.fuzz_factor != te_fuzz_init_factor) {
        t->cfg.fuzz_factor = te_fuzz_init_factor; /* fuzzing_init's factor (fuzzing.c:18) */
        t->dev_dirty = 1;
    }
    if (t->cfg.fuzz_seed && t->fz_seeded &&
        t->fz_gen != __atomic_load_n(&te_fuzz_init_gen, __ATOMIC_SEQ_CST))
        t->dev_dirty = 1; /* a fuzzing_init since the last upload re-seeds the state */
    if (t->cfg.slot_head != te_slot_head(&t->cfg)) { /* whatever set the config */
        t->cfg.slot_head = te_slot_head(&t->cfg);
        t->dev_dirty = 1;
    }
    {   /* the dst_modified carry, whatever set the config (post_args or setters) */
        const te_dev_cfg_t *c = &t->cfg;
        const uint32_t l2c = TE_DEC_ETH_ADDR(c->decoder) && c->encoder == TE_ENC_EN10MB &&
                             !(c->mac_mask & TE_MASK_DMAC1);
        if (l2c != c->l2carry) {
            t->cfg.l2carry = l2c;
            t->dev_dirty = 1;
        }
    }
    if (!t->dev_dirty && t->d_cfg)
        return 0;
    if (!t->d_cfg)
        HIPCHK(t, hipMalloc((void **)&t->d_cfg, sizeof(te_dev_cfg_t)));
    {   /* CIDR map entries past the inline lists: their spill lists go up with the config */
        const int32_t n[4] = {t->cfg.n_cidrmap1, t->cfg.n_cidrmap2, t->cfg.n_srcipmap, t->cfg.n_dstipmap};
        for (int w = 0; w < 4; w++) {
            const int32_t extra = n[w] > TE_MAX_CIDRMAP ? n[w] - TE_MAX_CIDRMAP : 0;
            t->cfg.cidr_spill[w] = 0;
            if (!extra)
                continue;
            if (!t->cspill[w]) {
                te_seterr(t, "CIDR map %d: %d entries past the inline list, none parsed", w, extra);
                return -1;
            }
            if (t->d_cspill_n[w] < extra) {
                hipFree(t->d_cspill[w]);
                t->d_cspill[w] = NULL;
                t->d_cspill_n[w] = 0;
                HIPCHK(t, hipMalloc((void **)&t->d_cspill[w], sizeof(te_cidrmap_t) * (size_t)extra));
                t->d_cspill_n[w] = extra;
            }
            HIPCHK(t, hipMemcpyAsync(t->d_cspill[w], t->cspill[w], sizeof(te_cidrmap_t) * (size_t)extra,
                                     hipMemcpyHostToDevice, t->stream));
            t->cfg.cidr_spill[w] = (uint64_t)(uintptr_t)t->d_cspill[w];
        }
    }
    HIPCHK(t, hipMemcpyAsync(t->d_cfg, &t->cfg, sizeof(te_dev_cfg_t), hipMemcpyHostToDevice, t->stream));
    if (t->portlut) {
        if (!t->d_portlut)
            HIPCHK(t, hipMalloc((void **)&t->d_portlut, 65536 * sizeof(uint16_t)));
        HIPCHK(t, hipMemcpyAsync(t->d_portlut, t->portlut, 65536 * sizeof(uint16_t), hipMemcpyHostToDevice,
                                 t->stream));
    }
    if (t->cfg.fuzz_seed) { /* fuzzing_init (fuzzing.c:12-20): the run-wide RNG state */
        const uint64_t gen = __atomic_load_n(&te_fuzz_init_gen, __ATOMIC_SEQ_CST);
        if (!t->d_fuzz_words)
            HIPCHK(t, hipMalloc((void **)&t->d_fuzz_words, 4 * sizeof(uint32_t)));
        if (!t->fz_seeded || t->fz_gen != gen) {
            /* seeded once per derivation (the tool's own fuzzing_init after post_args), and
               again by every explicit fuzzing_init call -- not on other config uploads, so
               the state carries across batches and tcpedit_packet calls */
            const uint32_t s0 = gen ? te_fuzz_init_seed : t->cfg.fuzz_seed;
            const uint32_t w[4] = {s0, s0, 0, 0};
            HIPCHK(t, hipMemcpyAsync(t->d_fuzz_words, w, sizeof(w), hipMemcpyHostToDevice, t->stream));
            t->fz_seeded = 1;
            t->fz_gen = gen;
        }
    }
    HIPCHK(t, hipStreamSynchronize(t->stream));
    t->dev_dirty = 0;
    t->cfg_gen++;
    return 0;
fail:
    return -1;
}

/* A batch over the pcap file header `hdr` (24 bytes) and the records `seg` (seg_len
 * bytes, whole records): a shard of a capture edited where it lies -- e.g. in the
 * caller's mmap of the file -- with no host copy (the index walk reads it in place, one
 * H2D copy puts header and records together in HBM).  tcpedit_batch_open is the same
 * over a whole image. */
static tcpedit_batch_t *batch_open(tcpedit_t *t, const uint8_t *hdr, const uint8_t *seg, size_t seg_len,
                                   const void *cache, size_t cache_len, uint64_t pkt_base, uint8_t *ng)
{
    const size_t len = 24 + seg_len;
    tcpedit_batch_t *b = calloc(1, sizeof(*b));
    if (!b) {
        te_seterr(t, "out of host memory");
        free(ng);
        return NULL;
    }
    b->ctx = t;
    b->pkt_base = pkt_base;
    /* index_image walks file offsets [24, len) of hdr + seg (the header from hdr, the
       records from seg) */
    if (index_image(t, b, hdr, seg, len) < 0)
        goto fail;
    if (b->linktype != (uint32_t)t->dlt) {
        te_seterr(t, "pcap linktype %u does not match the context DLT %d", b->linktype, t->dlt);
        goto fail;
    }
    if (te_upload_cfg(t) < 0)
        goto fail;
    HIPCHK(t, hipMalloc((void **)&b->d_in, len + 64));
    HIPCHK(t, hipMemcpyAsync(b->d_in, hdr, 24, hipMemcpyHostToDevice, t->stream));
    if (seg_len)
        HIPCHK(t, hipMemcpyAsync(b->d_in + 24, seg, seg_len, hipMemcpyHostToDevice, t->stream));
    HIPCHK(t, hipMalloc((void **)&b->d_out, b->out_cap + 64));
    HIPCHK(t, hipMalloc((void **)&b->d_status, b->n_pkts + 16));
    if (b->scratch_bytes)
        HIPCHK(t, hipMalloc((void **)&b->d_scratch, b->scratch_bytes));
    HIPCHK(t, hipMalloc((void **)&b->d_tiles, sizeof(te_tile_t) * (b->n_tiles + 1)));
    HIPCHK(t, hipMemcpyAsync(b->d_tiles, b->tiles, sizeof(te_tile_t) * b->n_tiles, hipMemcpyHostToDevice, t->stream));
    b->tcut_ok = 0;
    HIPCHK(t, hipMalloc((void **)&b->d_pkt_rel, sizeof(uint16_t) * (b->n_pkts + 1)));
    HIPCHK(t, hipMemcpyAsync(b->d_pkt_rel, b->pkt_rel, sizeof(uint16_t) * b->n_pkts, hipMemcpyHostToDevice,
                             t->stream));
    b->ws_bytes = WS_SLOTS(b->n_tiles) + 64;
    if (b->fast_kind == TE_FAST_WAVE)
        b->ws_bytes += 8 * TE_WK_SLOT_WORDS * (uint64_t)te_wave_grid();
    HIPCHK(t, hipMalloc((void **)&b->d_ws, b->ws_bytes));
    HIPCHK(t, hipMemsetAsync(b->d_ws, 0, b->ws_bytes, t->stream)); /* the list count starts at 0 */
    if (b->fast_tiles)
        HIPCHK(t, hipMalloc((void **)&b->d_tile_list, sizeof(uint32_t) * (b->n_tiles + 1)));
    b->q8_cap = (uint32_t)(b->n_pkts < TE_Q8_CAP ? b->n_pkts + 1 : TE_Q8_CAP);
    HIPCHK(t, hipMalloc((void **)&b->d_q8, 16 * (size_t)b->q8_cap));
    if (cache) {
        const uint8_t *cd;
        if (te_check_decoder_cfg(t, 1) < 0)
            goto fail;
        if (cache_data(t, (const uint8_t *)cache, cache_len, &cd, &b->dirbits_len) < 0)
            goto fail;
        HIPCHK(t, hipMalloc((void **)&b->d_dirbits, b->dirbits_len + 16));
        HIPCHK(t, hipMemcpyAsync(b->d_dirbits, cd, b->dirbits_len, hipMemcpyHostToDevice, t->stream));
    } else if (t->cfg.n_cidrmap1 && t->have[OPT_ENDPOINTS]) {
        te_seterr(t, "--endpoints requires a tcpprep cache file");
        goto fail;
    }
    HIPCHK(t, hipEventCreate(&b->ev0));
    HIPCHK(t, hipEventCreate(&b->ev1));
    HIPCHK(t, hipStreamSynchronize(t->stream));
    free(ng);
    return b;
fail:
    hipStreamSynchronize(t->stream);
    free(ng);
    tcpedit_batch_close(b);
    return NULL;
}

tcpedit_batch_t *tcpedit_batch_open(tcpedit_t *t, const void *pcap, size_t len, const void *cache, size_t cache_len,
                                    uint64_t pkt_base)
{
    if (!t || !pcap)
        return NULL;
    if (te_ensure_cfg(t) < 0)
        return NULL;
    uint8_t *ng = NULL; /* a pcapng image, as libpcap's reader delivers it (te_pcapng.c) */
    if (te_is_pcapng((const uint8_t *)pcap, len)) {
        char e[256];
        if (te_pcapng_to_pcap((const uint8_t *)pcap, len, &ng, &len, e, sizeof e) < 0) {
            te_seterr(t, "%s", e);
            return NULL;
        }
        pcap = ng;
    }
    if (len < 24) {
        te_seterr(t, "pcap image too short");
        free(ng);
        return NULL;
    }
    return batch_open(t, (const uint8_t *)pcap, (const uint8_t *)pcap + 24, len - 24, cache, cache_len, pkt_base,
                      ng);
}

tcpedit_batch_t *tcpedit_batch_open_segment(tcpedit_t *t, const void *hdr, const void *seg, size_t seg_len,
                                            const void *cache, size_t cache_len, uint64_t pkt_base)
{
    if (!t || !hdr || (!seg && seg_len))
        return NULL;
    if (te_ensure_cfg(t) < 0)
        return NULL;
    static const uint8_t none[1];
    return batch_open(t, (const uint8_t *)hdr, seg ? (const uint8_t *)seg : none, seg_len, cache, cache_len,
                      pkt_base, NULL);
}

/* TCPEDIT_HIP_NO_FAST=1 keeps every packet on the generic lane (A/B checks) */
static int fast_lane_off(void)
{
    const char *e = getenv("TCPEDIT_HIP_NO_FAST");
    return e && *e && *e != '0';
}

static int launch_ev(tcpedit_batch_t *b, int fixed_dir, hipEvent_t k0, hipEvent_t k1, int generic_only);

/* a window-mode launch (te_launch_t.win): the image's byte range and first record */
typedef struct te_win_req_s {
    uint64_t len, entry, entry_sub, base, limit;
    const uint64_t *entry_ptr;
    uint32_t nwin;
    /* the window-mode pipeline: the call's accumulator, the previous chunk's output image,
       the output image's device address when it is not the batch's (host-mapped) */
    uint64_t *acc;
    const uint8_t *prev_out;
    uint64_t head_max;
    uint8_t *out;
    uint64_t org;
} te_win_req_t;
/* the window workspace layout of d_win for `cap` windows: entries | exits | flags | bad | tot */
#define WIN_WS_BYTES(cap) (16ull * (cap) + 4ull * (cap) + 64)
/* the verdict word and the chain end, adjacent and 16-aligned: one 16-byte zeroing a launch
   (a fill that is not 16-aligned ran as two fill kernels, ~5 us each: a tenth of a C2 run) */
#define WIN_BAD_OFF(cap) ((20ull * (cap) + 15) & ~15ull)
#define WIN_TOT_OFF(cap) (WIN_BAD_OFF(cap) + 8)
static int launch(tcpedit_batch_t *b, int fixed_dir)
{
    return launch_ev(b, fixed_dir, NULL, NULL, 0);
}

/* the dst_modified carry's buffers for a launch over b (the context's word,
 * zeroed when first allocated: the reference's zeroed en10mb extra) */
/* DLT_JUNIPER_ETHER into an encoder that reads the decoder state (en10mb, user, hdlc; the
 * Juniper plugin's own encoder refuses every record, pppserial passes it through) */
static int jnpr_carry_cfg(const te_dev_cfg_t *c)
{
    return c->decoder == TE_DEC_JNPR &&
           (c->encoder == TE_ENC_EN10MB || c->encoder == TE_ENC_USER || c->encoder == TE_ENC_HDLC);
}

static int jctx_ready(tcpedit_t *t)
{
    if (t->d_jctx)
        return 0;
    if (hipMalloc((void **)&t->d_jctx, sizeof(te_jctx_t)) != hipSuccess ||
        hipMemsetAsync(t->d_jctx, 0, sizeof(te_jctx_t), t->stream) != hipSuccess) { /* TE_JC_NONE */
        t->d_jctx = NULL;
        te_seterr(t, "out of device memory (Juniper decoder state)");
        return -1;
    }
    return 0;
}

/* the Juniper decoder-state scan's buffers for a launch over b */
static int jnpr_bufs(tcpedit_t *t, tcpedit_batch_t *b, te_launch_t *L)
{
    if (b->n_pkts >= 0xffffffffull || jctx_ready(t) < 0)
        return -1;
    if (b->jnpr_cap < b->n_pkts) {
        hipFree(b->d_jnpr);
        hipFree(b->d_jtmp);
        b->d_jnpr = NULL;
        b->d_jtmp = NULL;
        b->jnpr_cap = 0;
        b->jtmp_bytes = te_l2carry_temp_bytes((uint32_t)b->n_pkts);
        if (!b->jtmp_bytes || hipMalloc((void **)&b->d_jnpr, 48 * (b->n_pkts + 1)) != hipSuccess ||
            hipMalloc(&b->d_jtmp, b->jtmp_bytes) != hipSuccess) {
            te_seterr(t, "out of device memory (Juniper decoder state)");
            return -1;
        }
        b->jnpr_cap = b->n_pkts;
    }
    L->n_pkts = (uint32_t)b->n_pkts;
    L->jscan = (uint64_t *)b->d_jnpr;
    L->jkeys = L->jscan + b->jnpr_cap + 1;
    L->jstates = (te_jstate_t *)(L->jkeys + b->jnpr_cap + 1);
    L->jctx = t->d_jctx;
    L->jtmp = b->d_jtmp;
    L->jtmp_bytes = b->jtmp_bytes;
    return 0;
}

static int l2carry_bufs(tcpedit_t *t, tcpedit_batch_t *b, te_launch_t *L)
{
    if (b->n_pkts >= 0xffffffffull)
        return -1;
    if (!t->d_l2word) {
        if (hipMalloc((void **)&t->d_l2word, sizeof(uint32_t)) != hipSuccess ||
            hipMemsetAsync(t->d_l2word, 0, sizeof(uint32_t), t->stream) != hipSuccess) {
            t->d_l2word = NULL;
            te_seterr(t, "out of device memory (dst_modified carry)");
            return -1;
        }
    }
    if (b->l2carry_cap < b->n_pkts) {
        hipFree(b->d_l2carry);
        hipFree(b->d_l2tmp);
        b->d_l2carry = NULL;
        b->d_l2tmp = NULL;
        b->l2carry_cap = 0;
        b->l2tmp_bytes = te_l2carry_temp_bytes((uint32_t)b->n_pkts);
        if (!b->l2tmp_bytes || hipMalloc((void **)&b->d_l2carry, 16 * (b->n_pkts + 1)) != hipSuccess ||
            hipMalloc(&b->d_l2tmp, b->l2tmp_bytes) != hipSuccess) {
            te_seterr(t, "out of device memory (dst_modified carry)");
            return -1;
        }
        b->l2carry_cap = b->n_pkts;
    }
    L->n_pkts = (uint32_t)b->n_pkts;
    L->l2carry = b->d_l2carry;
    L->l2carry_keys = b->d_l2carry + b->l2carry_cap + 1;
    L->l2carry_word = t->d_l2word;
    L->l2carry_tmp = b->d_l2tmp;
    L->l2carry_tmp_bytes = b->l2tmp_bytes;
    return 0;
}

/* generic_only: the generic pass over what the last (wave-lane) launch listed, under
 * that launch's parity -- for a run whose generic pass was left out by the hint */
/* the --mtu-trunc placement prediction for this tile cut (te_mtu_cuts), computed on the
   batch's stream the first time a cut is launched with this MTU; 0 when ready */
/* room for a placement prediction of this tile cut (d_tcut, d_tcut_raw) */
static int tcut_bufs(tcpedit_batch_t *b)
{
    if (b->tcut_cap < b->n_tiles + 1) {
        hipFree(b->d_tcut);
        hipFree(b->d_tcut_raw);
        b->d_tcut = NULL;
        b->d_tcut_raw = NULL;
        b->tcut_cap = 0;
        if (hipMalloc((void **)&b->d_tcut, sizeof(long long) * (b->n_tiles + 1)) != hipSuccess ||
            hipMalloc((void **)&b->d_tcut_raw, sizeof(long long) * ((b->n_tiles + 63) / 64 + 1)) != hipSuccess)
            return -1;
        b->tcut_cap = b->n_tiles + 1;
    }
    return 0;
}

static int mtu_cuts_ready(tcpedit_batch_t *b, int32_t mtu)
{
    tcpedit_t *t = b->ctx;
    if (b->tcut_ok && b->tcut_mtu == mtu)
        return 0;
    if (tcut_bufs(b) < 0)
        return -1;
    if (te_mtu_cuts(b->d_in, b->d_tiles, b->d_pkt_rel, (uint32_t)b->n_tiles, (uint32_t)mtu, b->d_tcut_raw, b->d_tcut,
                    t->stream) != 0)
        return -1;
    b->tcut_ok = 1;
    b->tcut_mtu = mtu;
    return 0;
}

static int launch_ev(tcpedit_batch_t *b, int fixed_dir, hipEvent_t k0, hipEvent_t k1, int generic_only)
{
    tcpedit_t *t = b->ctx;
    te_launch_t L;
    memset(&L, 0, sizeof(L));
    L.cfg = t->d_cfg;
    L.cfg_host = &t->cfg;
    L.portlut = t->cfg.has_portmap ? t->d_portlut : NULL;
    L.dirbits = b->d_dirbits;
    L.dirbits_len = b->dirbits_len;
    L.pkt_base = b->pkt_base;
    L.fixed_dir = fixed_dir;
    L.in = b->d_in;
    L.tiles = b->d_tiles;
    L.pkt_rel = b->d_pkt_rel;
    L.n_tiles = (uint32_t)b->n_tiles;
    L.in_swapped = (uint32_t)b->swapped;
    L.in_nsec = (uint32_t)b->nsec;
    L.out = b->d_out;
    L.out_base = b->out_base ? b->out_base : 24;
    L.tile_state = (uint64_t *)(b->d_ws + WS_STATE);
    L.ticket = (unsigned int *)(b->d_ws + WS_TICKET);
    L.status = b->d_status;
    L.counters = (uint64_t *)(b->d_ws + WS_COUNTERS);
    L.err = (uint64_t *)(b->d_ws + WS_ERR);
    L.scratch = b->d_scratch;
    L.zero_region = b->d_ws + WS_ZERO;
    L.zero_bytes = b->ws_bytes - WS_ZERO;
    L.grid = 0; /* resident blocks (CUs x occupancy) */
    L.slot_layout = b->slot_layout;
    /* size-preserving config: no edit step can change a record's length or drop
       it (efcs, VLAN add/del, fixlen, MTU truncation, skipped soft errors, and
       the reader's len < caplen trim are the only ways), so outputs sit at input offsets */
    const te_dev_cfg_t *c = &t->cfg;
    L.static_off = !b->slot_layout && static_capable(c) && !b->has_trim;
    L.rec0 = b->rec0 ? b->rec0 : 24;
    /* VLAN add as the only size change: every record grows by 4 bytes or is a hard error
       (dlt_en10mb_encode, en10mb.c:520-575), so outputs sit at input offset + 4 x index */
    L.static_grow = b->slot_layout && c->vlan == TE_VLAN_ADD && c->encoder == TE_ENC_EN10MB &&
                    c->decoder == TE_DEC_EN10MB && !c->efcs && c->fixlen == TE_FIXLEN_OFF &&
                    !c->mtu_truncate && !c->skip_soft_errors && !b->has_trim && !c->fuzz_seed &&
                    !(b->grow_off && b->grow_off_gen == t->cfg_gen) && !b->grow_never && !grow_off_env();
    /* a VLAN pop or --efcs as the only size change: outputs at input offset - 4 x index
       (checked record by record like static_grow) */
    L.static_shrink = !b->slot_layout && !b->has_trim && !b->swapped && !b->nsec &&
                              !(b->grow_off && b->grow_off_gen == t->cfg_gen) && !b->grow_never && !grow_off_env()
                          ? static_shrink_kind(c)
                          : TE_SZ_NONE;
    L.grow_bad = (uint32_t *)(b->d_ws + WS_GROW_BAD);
    b->last_grow = L.static_grow ? 4 : L.static_shrink ? -4 : 0;
    /* --mtu-trunc on the wave lane: tiles placed by the predicted cuts (fast_capable_mtu) */
    L.static_mtu = b->mtu_fast && b->fast_kind == TE_FAST_WAVE && fast_capable_mtu(c) && !b->slot_layout &&
                   !b->has_trim && !b->swapped && !b->nsec && !b->dirbits_len && b->n_tiles > 0 &&
                   !(b->grow_off && b->grow_off_gen == t->cfg_gen) && !b->grow_never && !grow_off_env() &&
                   !fast_lane_off() && mtu_cuts_ready(b, c->mtu) == 0;
    L.tcut = L.static_mtu ? b->d_tcut : NULL;
    L.mtu = (uint32_t)c->mtu;
    b->last_mtu = L.static_mtu;
    /* --fuzz-seed on the wave lane: tiles placed by the predicted cuts, which the launch
       computes after drawing the states (fast_capable_fuzz) */
    L.static_fz = b->fz_fast && b->fast_kind == TE_FAST_WAVE && fast_capable_fuzz(c) && !b->slot_layout &&
                  !b->has_trim && !b->swapped && !b->nsec && !b->d_dirbits && b->n_tiles > 0 && b->n_pkts > 0 &&
                  !b->fuzz_probe_only && !b->q18_only && !(b->grow_off && b->grow_off_gen == t->cfg_gen) && !b->grow_never &&
                  !grow_off_env() && !fast_lane_off() && tcut_bufs(b) == 0;
    if (L.static_fz) {
        const uint64_t words = b->n_tiles + 1 + b->n_pkts; /* the reach list, its count, a word a record */
        if (b->fzlist_cap < words) {
            hipFree(b->d_fzlist);
            b->d_fzlist = NULL;
            b->fzlist_cap = 0;
            if (hipMalloc((void **)&b->d_fzlist, 4 * words) != hipSuccess)
                return -1;
            b->fzlist_cap = words;
        }
        L.tcut = b->d_tcut;
        L.tcut_raw = b->d_tcut_raw;
        L.fz_list = b->d_fzlist;
        b->tcut_ok = 0; /* (d_tcut now holds this launch's fuzz cuts) */
    }
    b->last_fz = L.static_fz;
    L.fast = b->fast_tiles && !fast_lane_off() &&
             ((L.static_off && fast_capable(c)) || (L.static_grow && fast_capable_grow(c)) ||
              (L.static_shrink && fast_capable_shrink(c)) || L.static_mtu || L.static_fz);
    L.fast_v6 = fast_v6_ok(c);
    /* a batch whose input + output outgrow the 256 MiB Infinity Cache streams through it:
       nontemporal loads and stores (TCPEDIT_HIP_STREAM=0/1 overrides, for A/B runs) */
    {
        const char *e = getenv("TCPEDIT_HIP_STREAM");
        L.stream = e && *e ? atoi(e) != 0 : (b->in_len + b->out_cap) > ((uint64_t)256 << 20);
    }
    L.fast_kind = b->fast_kind;
    L.wk_small = b->wk_small;
    L.slots = (uint64_t *)(b->d_ws + WS_SLOTS(b->n_tiles));
    if (L.fast && b->gen_hint_ok && b->gen_hint_gen == t->cfg_gen)
        L.grid = b->last_listed ? (int)b->last_listed : 1; /* the generic kernel's grid after the fast lane */
    L.tile_list = b->d_tile_list;
    L.list_cnt = (uint32_t *)(b->d_ws + WS_LIST_CNT(b->n_tiles));
    L.parity = (uint32_t)(generic_only ? (b->launches - 1) & 1 : b->launches++ & 1);
    b->last_fast = L.fast;
    b->last_cnt_off = L.fast && L.parity ? WS_COUNTERS1 : WS_COUNTERS;
    L.counters = (uint64_t *)(b->d_ws + b->last_cnt_off);
    L.counters_next = (uint64_t *)(b->d_ws + (b->last_cnt_off == WS_COUNTERS ? WS_COUNTERS1 : WS_COUNTERS));
    L.ws_zero = (uint64_t *)(b->d_ws + WS_ZERO);
    L.ev_k0 = k0;
    L.ev_k1 = k1;
    L.generic_only = generic_only;
    L.q8_list = b->d_q8;
    L.q8_cap = b->d_q8 ? b->q8_cap : 0;
    /* wave lane: this batch's previous run under this config listed nothing, so the
       generic pass is left out (batch_run_dir runs it after all if a run does list) */
    L.skip_generic = !generic_only && L.fast && b->fast_kind == TE_FAST_WAVE && b->gen_hint_ok &&
                     b->gen_hint_gen == t->cfg_gen && b->last_listed == 0;
    if (generic_only)
        L.grid = b->last_listed ? (int)b->last_listed : 1;
    if (c->fuzz_seed && (!L.fast || L.static_fz) && b->n_pkts) {
        /* --fuzz-seed: room for a state per record and a word per 1024 records */
        const uint64_t need = b->n_pkts;
        if (b->fuzz_cap < need) {
            hipFree(b->d_fuzz);
            b->d_fuzz = NULL;
            b->fuzz_cap = 0;
            if (hipMalloc((void **)&b->d_fuzz, 4 * (need + need / 1024 + 2)) != hipSuccess)
                return -1;
            b->fuzz_cap = need;
        }
        if (b->n_pkts > 0xffffffffull || !t->d_fuzz_words)
            return -1;
        L.fuzz_states = b->d_fuzz;
        L.fuzz_blk = b->d_fuzz + b->fuzz_cap + 1;
        L.fuzz_words = t->d_fuzz_words;
        L.n_pkts = (uint32_t)b->n_pkts;
        L.fuzz_probe_only = b->fuzz_probe_only;
        L.q18_only = b->q18_only;
    }
    if (c->l2carry && !L.fast && b->n_pkts && l2carry_bufs(t, b, &L) < 0)
        return -1;
    if (jnpr_carry_cfg(c) && !L.fast && b->n_pkts && jnpr_bufs(t, b, &L) < 0)
        return -1;
    L.any_dec = c->decoder != TE_DEC_EN10MB || c->encoder == TE_ENC_NOENC || c->encoder == TE_ENC_PPP;
    if (b->win_req) { /* window mode: the wave lane finds the records (no tiles, no index) */
        const te_win_req_t *q = b->win_req;
        L.win = 1;
        L.win_len = q->len;
        L.win_entry = q->entry;
        L.win_entry_ptr = q->entry_ptr;
        L.win_entry_sub = q->entry_sub;
        L.win_base = q->base;
        L.win_limit = q->limit;
        L.nwin = q->nwin;
        L.w_entry = (uint64_t *)b->d_win;
        L.w_exit = L.w_entry + b->win_cap;
        L.w_flags = (uint32_t *)(L.w_exit + b->win_cap);
        L.win_bad = (uint32_t *)(b->d_win + WIN_BAD_OFF(b->win_cap));
        L.win_tot = (uint64_t *)(b->d_win + WIN_TOT_OFF(b->win_cap));
        L.win_acc = q->acc;
        L.win_prev_out = q->prev_out;
        L.win_head_max = q->head_max;
        L.win_org = q->org;
        if (q->out)
            L.out = q->out;
        L.slots = (uint64_t *)(b->d_ws + WS_SLOTS(b->n_tiles));
        L.stream = (b->in_len + b->out_cap) > ((uint64_t)256 << 20);
    }
    const int rc = te_launch_edit(&L, t->stream);
    if (!generic_only) {
        b->last_skipped = L.skip_generic;
        b->last_fgrid = (L.fast && b->fast_kind == TE_FAST_WAVE) || L.win ? L.out_fgrid : 0;
    }
    return rc;
}

/* the output file header: pcap_open_dead(out_dlt, 65535) + pcap_dump_open
   (tcprewrite.c:124,147), LE microsecond, linktype = the encoder's output DLT */
static void out_header(const tcpedit_t *t, uint8_t *h)
{
    static const uint8_t base[24] = {0xd4, 0xc3, 0xb2, 0xa1, 2, 0, 4, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                     0xff, 0xff, 0, 0, 1, 0, 0, 0};
    memcpy(h, base, 24);
    /* pcap_dump_open writes dlt_to_linktype(dlt): DLT_RAW (12) is LINKTYPE_RAW (101) */
    const uint32_t lt = t->cfg.out_linktype == 12 ? 101u : (uint32_t)t->cfg.out_linktype;
    memcpy(h + 20, &lt, 4);
}

/* te_q8_replay over what the last launch of `b` listed, on `st`.
 * file_start: the batch's first record is the capture's first (the reference's buffer
 * starts zeroed there); init: the initial buffer instead (tcpedit_packet). */
static int run_q8(tcpedit_t *t, tcpedit_batch_t *b, int fixed_dir, int file_start, const uint8_t *d_init,
                  uint32_t init_len, hipStream_t st)
{
    if (!t->d_q8_scratch) {
        if (hipMalloc((void **)&t->d_q8_scratch, (size_t)TE_Q8_THREADS * te_q8_slot_bytes()) != hipSuccess) {
            t->d_q8_scratch = NULL;
            te_seterr(t, "out of device memory (stale-buffer replay scratch)");
            return -1;
        }
    }
    te_launch_t L;
    memset(&L, 0, sizeof(L));
    L.cfg = t->d_cfg;
    L.cfg_host = &t->cfg;
    L.portlut = t->cfg.has_portmap ? t->d_portlut : NULL;
    L.dirbits = b->d_dirbits;
    L.dirbits_len = b->dirbits_len;
    L.pkt_base = b->pkt_base;
    L.fixed_dir = fixed_dir;
    L.in = b->d_in;
    L.tiles = b->d_tiles;
    L.pkt_rel = b->d_pkt_rel;
    L.n_tiles = (uint32_t)b->n_tiles;
    L.in_swapped = (uint32_t)b->swapped;
    L.in_nsec = (uint32_t)b->nsec;
    L.out = b->d_out;
    L.out_base = b->out_base ? b->out_base : 24;
    L.rec0 = b->rec0 ? b->rec0 : 24;
    L.status = b->d_status;
    L.counters = (uint64_t *)(b->d_ws + b->last_cnt_off);
    L.err = (uint64_t *)(b->d_ws + WS_ERR);
    L.q8_list = b->d_q8;
    L.q8_cap = b->q8_cap;
    L.q8_scratch = t->d_q8_scratch;
    L.q8_threads = TE_Q8_THREADS;
    L.q8_file_start = file_start;
    L.q8_init = d_init;
    L.q8_init_len = init_len;
    if (b->pre_staged && b->npre) {
        L.q8_pre = b->d_pre;
        L.q8_pre_off = b->d_pre_off;
        L.q8_npre = b->npre;
        L.q8_pre_file_start = b->pre_file_start;
    }
    if (t->cfg.fuzz_seed && b->d_fuzz && (!b->last_fast || b->last_fz))
        L.fuzz_states = b->d_fuzz;
    if (t->cfg.l2carry && !b->last_fast)
        L.l2carry = b->d_l2carry; /* the last launch's scan: each replayed record's carried value */
    if (jnpr_carry_cfg(&t->cfg) && !b->last_fast && b->d_jnpr && b->jnpr_cap >= b->n_pkts) {
        /* ... and each replayed record's Juniper decoder state (the context's word now holds
           the launch's last: a record with none before it in the launch is not replayed) */
        L.jscan = (uint64_t *)b->d_jnpr;
        L.jstates = (te_jstate_t *)(L.jscan + 2 * (b->jnpr_cap + 1));
        L.jctx = t->d_jctx;
    }
    if (te_launch_q8(&L, st) != 0) {
        te_seterr(t, "stale-buffer replay launch failed: %s", hipGetErrorString(hipGetLastError()));
        return -1;
    }
    return 0;
}

int tcpedit_batch_set_prefix(tcpedit_t *t, tcpedit_batch_t *b, const void *recs, size_t len)
{
    if (!t || !b || (len && !recs))
        return TCPEDIT_ERROR;
    b->pre_host = len ? (const uint8_t *)recs : NULL;
    b->pre_len = len;
    b->pre_staged = 0;
    b->npre = 0;
    return TCPEDIT_OK;
}

/* the prefix's last records (up to TE_Q8_PRE_RECS / TE_Q8_PRE_BYTES) to the device: a
 * forward walk of its headers (the chain only runs forward), keeping a ring of offsets */
static int stage_prefix(tcpedit_t *t, tcpedit_batch_t *b)
{
    const uint8_t *r = b->pre_host;
    const size_t len = b->pre_len;
    uint64_t *ring = malloc(sizeof(uint64_t) * TE_Q8_PRE_RECS);
    if (!ring) {
        te_seterr(t, "out of memory");
        return -1;
    }
    uint64_t n = 0;
    size_t p = 0;
    while (p + 16 <= len) {
        const uint32_t cl = rd32(r + p + 8, b->swapped);
        if (cl > 262144u || p + 16 + cl > len)
            break;
        ring[n++ % TE_Q8_PRE_RECS] = p;
        p += 16 + (size_t)cl;
    }
    if (p != len) {
        free(ring);
        te_seterr(t, "tcpedit_batch_set_prefix: the records do not end where the batch starts (byte %zu of %zu)", p,
                  len);
        return -1;
    }
    /* the newest records that fit the limits */
    uint64_t k = n < TE_Q8_PRE_RECS ? n : TE_Q8_PRE_RECS;
    while (k > 1 && len - ring[(n - k) % TE_Q8_PRE_RECS] > TE_Q8_PRE_BYTES)
        k--;
    const uint64_t first = n - k, lo = k ? ring[first % TE_Q8_PRE_RECS] : len;
    uint64_t *off = malloc(sizeof(uint64_t) * (k ? k : 1));
    if (!off) {
        free(ring);
        te_seterr(t, "out of memory");
        return -1;
    }
    for (uint64_t i = 0; i < k; i++)
        off[i] = ring[(first + i) % TE_Q8_PRE_RECS] - lo;
    free(ring);
    hipFree(b->d_pre);
    hipFree(b->d_pre_off);
    b->d_pre = NULL;
    b->d_pre_off = NULL;
    if (hipMalloc((void **)&b->d_pre, (len - lo) + 64) != hipSuccess ||
        hipMalloc((void **)&b->d_pre_off, sizeof(uint64_t) * (k ? k : 1)) != hipSuccess ||
        hipMemcpyAsync(b->d_pre, r + lo, len - lo, hipMemcpyHostToDevice, t->stream) != hipSuccess ||
        hipMemcpyAsync(b->d_pre_off, off, sizeof(uint64_t) * k, hipMemcpyHostToDevice, t->stream) != hipSuccess ||
        hipStreamSynchronize(t->stream) != hipSuccess) {
        free(off);
        te_seterr(t, "out of device memory (prefix records)");
        return -1;
    }
    free(off);
    b->npre = (uint32_t)k;
    /* the prefix's first record is record pkt_base - n of the job: the capture's first when 0 */
    b->pre_file_start = first == 0 && b->pkt_base == n;
    b->pre_staged = 1;
    return 0;
}

/* after a run whose replay failed a record: with a prefix set, stage it and replay the
 * listed records again (idempotent for the ones already replayed), counters re-read */
static int retry_q8_with_prefix(tcpedit_t *t, tcpedit_batch_t *b, int fixed_dir, uint64_t *counters)
{
    if (!b->pre_host || b->pre_staged)
        return 0;
    if (stage_prefix(t, b) < 0)
        return -1;
    HIPCHK(t, hipMemsetAsync(b->d_ws + b->last_cnt_off + 8 * TE_CNT_Q8_FAILED, 0, 8, t->stream));
    if (run_q8(t, b, fixed_dir, b->pkt_base == 0, NULL, 0, t->stream) < 0)
        return -1;
    HIPCHK(t, hipMemcpyAsync(counters, b->d_ws + b->last_cnt_off, sizeof(b->counters), hipMemcpyDeviceToHost,
                             t->stream));
    HIPCHK(t, hipStreamSynchronize(t->stream));
    return 0;
fail:
    return -1;
}

static int batch_run_dir(tcpedit_t *t, tcpedit_batch_t *b, int fixed_dir)
{
    float ms = 0;
    if (te_upload_cfg(t) < 0)
        return TCPEDIT_ERROR;
    /* pcap_open_dead(out_dlt, 65535) + pcap_dump_open (tcprewrite.c:124,147) */
    out_header(t, b->ohdr);
    HIPCHK(t, hipMemcpyAsync(b->d_out, b->ohdr, 24, hipMemcpyHostToDevice, t->stream));
    HIPCHK(t, hipEventRecord(b->ev0, t->stream));
    if (launch(b, fixed_dir) != 0) {
        te_seterr(t, "kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
        return TCPEDIT_ERROR;
    }
    HIPCHK(t, hipEventRecord(b->ev1, t->stream));
    HIPCHK(t, hipMemcpyAsync(b->counters, b->d_ws + b->last_cnt_off, sizeof(b->counters), hipMemcpyDeviceToHost,
                             t->stream));
    HIPCHK(t, hipMemcpyAsync(b->err, b->d_ws + WS_ERR, sizeof(b->err), hipMemcpyDeviceToHost, t->stream));
    if (b->last_fast)
        HIPCHK(t, hipMemcpyAsync(&b->last_listed, b->d_ws + WS_LIST_CNT(b->n_tiles) + 4 * ((b->launches - 1) & 1),
                                 sizeof(uint32_t), hipMemcpyDeviceToHost, t->stream));
    if (b->last_fgrid) {
        if (!b->slots_host)
            b->slots_host = malloc(8 * TE_WK_SLOT_WORDS * (size_t)te_wave_grid());
        HIPCHK(t, hipMemcpyAsync(b->slots_host, b->d_ws + WS_SLOTS(b->n_tiles),
                                 8 * TE_WK_SLOT_WORDS * (size_t)b->last_fgrid, hipMemcpyDeviceToHost, t->stream));
    }
    if (b->last_grow || b->last_mtu || b->last_fz)
        HIPCHK(t, hipMemcpyAsync(&b->grow_bad, b->d_ws + WS_GROW_BAD, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                 t->stream));
    HIPCHK(t, hipStreamSynchronize(t->stream));
    if (b->last_fast && b->last_skipped && b->last_listed) {
        /* the hint was wrong (it can be after tcpedit_batch_update_input): run the generic
           pass now and read the counters, error and violation words again -- before the
           static-placement check below, since the tiles it edits can break that placement */
        if (launch_ev(b, fixed_dir, NULL, NULL, 1) != 0) {
            te_seterr(t, "kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
            return TCPEDIT_ERROR;
        }
        HIPCHK(t, hipMemcpyAsync(b->counters, b->d_ws + b->last_cnt_off, sizeof(b->counters),
                                 hipMemcpyDeviceToHost, t->stream));
        HIPCHK(t, hipMemcpyAsync(b->err, b->d_ws + WS_ERR, sizeof(b->err), hipMemcpyDeviceToHost, t->stream));
        if (b->last_grow || b->last_mtu || b->last_fz) /* the listed tiles can break static placement too */
            HIPCHK(t, hipMemcpyAsync(&b->grow_bad, b->d_ws + WS_GROW_BAD, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                     t->stream));
        HIPCHK(t, hipStreamSynchronize(t->stream));
        b->last_skipped = 0;
    }
    if ((b->last_grow || b->last_mtu || b->last_fz) && b->grow_bad) {
        /* a record did not grow by exactly 4 bytes (a tile's --mtu-trunc or fuzz cut was not
           the predicted one): place this batch by scan + look-back from now on, and run it
           again that way -- from the RNG state this run started at (te_fuzz_scan kept it in
           words[1]) */
        if (b->last_fz)
            HIPCHK(t, hipMemcpyAsync(t->d_fuzz_words, t->d_fuzz_words + 1, sizeof(uint32_t), hipMemcpyDeviceToDevice,
                                     t->stream));
        b->grow_off = 1;
        b->grow_off_gen = t->cfg_gen;
        b->grow_bad = 0;
        if (launch(b, fixed_dir) != 0) {
            te_seterr(t, "kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
            return TCPEDIT_ERROR;
        }
        HIPCHK(t, hipEventRecord(b->ev1, t->stream));
        HIPCHK(t, hipMemcpyAsync(b->counters, b->d_ws + b->last_cnt_off, sizeof(b->counters),
                                 hipMemcpyDeviceToHost, t->stream));
        HIPCHK(t, hipMemcpyAsync(b->err, b->d_ws + WS_ERR, sizeof(b->err), hipMemcpyDeviceToHost, t->stream));
        HIPCHK(t, hipStreamSynchronize(t->stream));
    }
    if (b->counters[TE_CNT_UNSUPPORTED] && !b->q8_defer) {
        /* records whose edit read the reference's stale static buffer: replay them */
        if (run_q8(t, b, fixed_dir, b->pkt_base == 0, NULL, 0, t->stream) < 0)
            return TCPEDIT_ERROR;
        HIPCHK(t, hipMemcpyAsync(b->counters, b->d_ws + b->last_cnt_off, sizeof(b->counters),
                                 hipMemcpyDeviceToHost, t->stream));
        HIPCHK(t, hipStreamSynchronize(t->stream));
        /* bytes from before the batch: walk back into the records the caller staged */
        if (b->counters[TE_CNT_Q8_FAILED] && retry_q8_with_prefix(t, b, fixed_dir, b->counters) < 0)
            return TCPEDIT_ERROR;
    }
    for (int i = 0; i < b->last_fgrid; i++) { /* the wave lane's per-block totals */
        const uint64_t *v = b->slots_host + TE_WK_SLOT_WORDS * (size_t)i;
        b->counters[TE_CNT_PACKETS] += v[0];
        b->counters[TE_CNT_WRITTEN] += v[0] - v[4]; /* (fuzz drops) */
        b->counters[TE_CNT_BYTES_IN] += v[1];
        b->counters[TE_CNT_BYTES_OUT] += v[1] + (uint64_t)((int64_t)b->last_grow * (int64_t)v[0]) /* +- 4 a record */
                                         - v[3];                                        /* the MTU / fuzz cuts */
        b->counters[TE_CNT_EDITED] += v[2];
        b->counters[TE_CNT_SOFT] += v[5];
    }
    if (b->last_fast) { /* same batch + same config lists the same tiles next time */
        b->gen_hint_ok = 1;
        b->gen_hint_gen = t->cfg_gen;
    }
    b->err[0] = ~b->err[0]; /* stored complemented (0 = no error -> ~0) */
    b->err[1] = ~b->err[1];
    HIPCHK(t, hipEventElapsedTime(&ms, b->ev0, b->ev1));
    b->kernel_ms = ms;
    b->ran = 1;
    b->status_valid = 0;
    if (b->err[2]) {
        te_seterr(t, "device look-back timed out (%llu tiles)", (unsigned long long)b->err[2]);
        return TCPEDIT_ERROR;
    }
    t->pub.runtime.packetnum += b->counters[TE_CNT_PACKETS];
    t->pub.runtime.total_bytes += b->counters[TE_CNT_BYTES_OUT];
    t->pub.runtime.pkts_edited += b->counters[TE_CNT_EDITED];
    return TCPEDIT_OK;
fail:
    return TCPEDIT_ERROR;
}

/* host copy of tcpr_random's LCG advanced by k steps (te_fuzz_states does the same on
   the device) */
static uint32_t lcg_jump_host(uint32_t x, uint64_t k)
{
    uint32_t am = 1, ap = 0, cm = 1103515245u, cp = 12345u;
    for (; k; k >>= 1) {
        if (k & 1) {
            am *= cm;
            ap = ap * cm + cp;
        }
        cp = (cm + 1u) * cp;
        cm *= cm;
    }
    return am * x + ap;
}

int64_t tcpedit_batch_fuzz_reach(tcpedit_t *t, tcpedit_batch_t *b)
{
    if (!t || !b)
        return TCPEDIT_ERROR;
    if (te_upload_cfg(t) < 0)
        return TCPEDIT_ERROR;
    if (!t->cfg.fuzz_seed || !b->n_pkts)
        return 0;
    uint32_t w[4];
    b->fuzz_probe_only = 1;
    const int rc = launch(b, -1);
    b->fuzz_probe_only = 0;
    if (rc != 0) {
        te_seterr(t, "kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
        return TCPEDIT_ERROR;
    }
    HIPCHK(t, hipMemcpyAsync(w, t->d_fuzz_words, sizeof(w), hipMemcpyDeviceToHost, t->stream));
    HIPCHK(t, hipStreamSynchronize(t->stream));
    return (int64_t)w[2];
fail:
    return TCPEDIT_ERROR;
}

/* SURVEY Q18 across shards: the dst_modified value the batch's last C2S writer leaves (0
 * or 1), or 2 when no record of the batch writes it (the carry passes through unchanged)
 * -- found by the carry's own mark + scan, before any edit, so that the ranks of a sharded
 * job can exchange it and each seed its context with the nearest earlier shard's value
 * (tcpedit_set_l2carry).  2 as well for a config without the carry. */
int tcpedit_batch_l2carry_out(tcpedit_t *t, tcpedit_batch_t *b)
{
    if (!t || !b)
        return TCPEDIT_ERROR;
    if (te_upload_cfg(t) < 0)
        return TCPEDIT_ERROR;
    if (!t->cfg.l2carry || !b->n_pkts)
        return 2;
    uint64_t last = 0;
    if (t->cfg.fuzz_seed) {
        /* a fuzzed record's second encode writes the carry too: the fuzz states first (from
           the context's running start -- the earlier shards' draws skipped already), then
           the carry's mark run of the edit and its scan (te_launch_edit, q18_only) */
        b->q18_only = 1;
        const int rc = launch(b, -1);
        b->q18_only = 0;
        if (rc != 0) {
            te_seterr(t, "dst_modified carry launch failed: %s", hipGetErrorString(hipGetLastError()));
            return TCPEDIT_ERROR;
        }
        HIPCHK(t, hipMemcpyAsync(&last, b->d_l2carry + b->n_pkts, sizeof(last), hipMemcpyDeviceToHost, t->stream));
        HIPCHK(t, hipStreamSynchronize(t->stream));
        if (last >> 63) {
            te_seterr(t, "dst_modified carry: a fuzzed record's second encode read stale buffer bytes (not served)");
            return TCPEDIT_ERROR;
        }
        return (last >> 1) ? (int)(last & 1u) : 2;
    }
    te_launch_t L;
    memset(&L, 0, sizeof(L));
    L.cfg = t->d_cfg;
    L.cfg_host = &t->cfg;
    L.dirbits = b->d_dirbits;
    L.dirbits_len = b->dirbits_len;
    L.pkt_base = b->pkt_base;
    L.fixed_dir = -1;
    L.in = b->d_in;
    L.tiles = b->d_tiles;
    L.pkt_rel = b->d_pkt_rel;
    L.n_tiles = (uint32_t)b->n_tiles;
    L.in_swapped = (uint32_t)b->swapped;
    L.in_nsec = (uint32_t)b->nsec;
    if (l2carry_bufs(t, b, &L) < 0 || (jnpr_carry_cfg(&t->cfg) && jnpr_bufs(t, b, &L) < 0))
        return TCPEDIT_ERROR;
    if (te_launch_l2carry(&L, t->stream) != 0) {
        te_seterr(t, "dst_modified carry launch failed: %s", hipGetErrorString(hipGetLastError()));
        return TCPEDIT_ERROR;
    }
    HIPCHK(t, hipMemcpyAsync(&last, L.l2carry + b->n_pkts, sizeof(last), hipMemcpyDeviceToHost, t->stream));
    HIPCHK(t, hipStreamSynchronize(t->stream));
    return (last >> 1) ? (int)(last & 1u) : 2; /* position 0 is the context's own word */
fail:
    return TCPEDIT_ERROR;
}

/* seed the context's dst_modified carry as an earlier shard left it */
int tcpedit_set_l2carry(tcpedit_t *t, int value)
{
    if (!t || value < 0 || value > 1)
        return TCPEDIT_ERROR;
    if (te_upload_cfg(t) < 0)
        return TCPEDIT_ERROR;
    if (!t->d_l2word)
        HIPCHK(t, hipMalloc((void **)&t->d_l2word, sizeof(uint32_t)));
    const uint32_t w = (uint32_t)value;
    HIPCHK(t, hipMemcpyAsync(t->d_l2word, &w, sizeof(w), hipMemcpyHostToDevice, t->stream));
    HIPCHK(t, hipStreamSynchronize(t->stream));
    return TCPEDIT_OK;
fail:
    return TCPEDIT_ERROR;
}

/* DLT_JUNIPER_ETHER across shards: the decoder state the batch's last whole inner decode
 * leaves (TCPEDIT_JNPR_STATE_BYTES into `state`), found by the state scan before any edit;
 * 1 when the batch has such a decode, 0 when none (the carry passes through), also for a
 * config without the carry.  A whole decode reads no carried state, so the ranks of a
 * sharded job can exchange these first and seed each context with the nearest earlier
 * shard's (tcpedit_set_jnpr_state) before the Q18 carry-out, which reads it. */
int tcpedit_batch_jnpr_out(tcpedit_t *t, tcpedit_batch_t *b, void *state, size_t len)
{
    if (!t || !b || !state || len < sizeof(te_jctx_t))
        return TCPEDIT_ERROR;
    memset(state, 0, sizeof(te_jctx_t));
    if (te_upload_cfg(t) < 0)
        return TCPEDIT_ERROR;
    if (!jnpr_carry_cfg(&t->cfg) || !b->n_pkts)
        return 0;
    te_launch_t L;
    memset(&L, 0, sizeof(L));
    L.cfg = t->d_cfg;
    L.cfg_host = &t->cfg;
    L.dirbits = b->d_dirbits;
    L.dirbits_len = b->dirbits_len;
    L.pkt_base = b->pkt_base;
    L.fixed_dir = -1;
    L.in = b->d_in;
    L.tiles = b->d_tiles;
    L.pkt_rel = b->d_pkt_rel;
    L.n_tiles = (uint32_t)b->n_tiles;
    L.in_swapped = (uint32_t)b->swapped;
    L.in_nsec = (uint32_t)b->nsec;
    te_jctx_t *d_out = NULL;
    te_jctx_t h;
    if (jnpr_bufs(t, b, &L) < 0)
        return TCPEDIT_ERROR;
    HIPCHK(t, hipMalloc((void **)&d_out, sizeof(te_jctx_t)));
    if (te_launch_jnpr(&L, d_out, t->stream) != 0) {
        te_seterr(t, "Juniper decoder-state launch failed: %s", hipGetErrorString(hipGetLastError()));
        hipFree(d_out);
        return TCPEDIT_ERROR;
    }
    HIPCHK(t, hipMemcpyAsync(&h, d_out, sizeof(h), hipMemcpyDeviceToHost, t->stream));
    HIPCHK(t, hipStreamSynchronize(t->stream));
    hipFree(d_out);
    memcpy(state, &h, sizeof(h));
    return h.valid == TE_JC_VALID ? 1 : 0;
fail:
    hipFree(d_out);
    return TCPEDIT_ERROR;
}

/* seed the context's Juniper decoder state as an earlier shard left it: `state` from
 * tcpedit_batch_jnpr_out (1 returned there), or NULL for none before (the capture's start);
 * unknown = 1 marks it not known (a frame that needs it then fails loudly) */
int tcpedit_set_jnpr_state(tcpedit_t *t, const void *state, size_t len, int unknown)
{
    if (!t || (state && len < sizeof(te_jctx_t)))
        return TCPEDIT_ERROR;
    if (te_upload_cfg(t) < 0 || jctx_ready(t) < 0)
        return TCPEDIT_ERROR;
    te_jctx_t h;
    memset(&h, 0, sizeof(h));
    if (state) {
        memcpy(&h, state, sizeof(h));
        if (h.valid != TE_JC_VALID && h.valid != TE_JC_NONE) {
            te_seterr(t, "not a Juniper decoder state");
            return TCPEDIT_ERROR;
        }
    }
    if (unknown)
        h.valid = TE_JC_UNKNOWN;
    HIPCHK(t, hipMemcpyAsync(t->d_jctx, &h, sizeof(h), hipMemcpyHostToDevice, t->stream));
    HIPCHK(t, hipStreamSynchronize(t->stream));
    return TCPEDIT_OK;
fail:
    return TCPEDIT_ERROR;
}

int tcpedit_fuzz_skip(tcpedit_t *t, uint64_t draws)
{
    if (!t)
        return TCPEDIT_ERROR;
    if (te_upload_cfg(t) < 0)
        return TCPEDIT_ERROR;
    if (!t->cfg.fuzz_seed || !draws)
        return TCPEDIT_OK;
    uint32_t w[4];
    HIPCHK(t, hipMemcpyAsync(w, t->d_fuzz_words, sizeof(w), hipMemcpyDeviceToHost, t->stream));
    HIPCHK(t, hipStreamSynchronize(t->stream));
    w[0] = lcg_jump_host(w[0], 3 * draws); /* tcpr_random = three LCG steps (utils.c:436-458) */
    HIPCHK(t, hipMemcpyAsync(t->d_fuzz_words, w, sizeof(w), hipMemcpyHostToDevice, t->stream));
    HIPCHK(t, hipStreamSynchronize(t->stream));
    return TCPEDIT_OK;
fail:
    return TCPEDIT_ERROR;
}

const uint8_t *tcpedit_batch_status(tcpedit_batch_t *b)
{
    if (!b || !b->ran)
        return NULL;
    if (!b->status_valid) {
        if (!b->status)
            b->status = malloc(b->n_pkts + 1);
        if (hipMemcpy(b->status, b->d_status, b->n_pkts, hipMemcpyDeviceToHost) != hipSuccess)
            return NULL;
        b->status_valid = 1;
    }
    return b->status;
}

/* new bytes for a batch's records, in place: the same file header and record headers (so
 * the index stands), other record bytes -- tcpreplay-edit's --preload-pcap cache, edited
 * from pass to pass (te_replay.c) */
int tcpedit_batch_update_input(tcpedit_t *t, tcpedit_batch_t *b, const void *img, size_t len)
{
    if (!t || !b || !img || len != b->in_len)
        return TCPEDIT_ERROR;
    HIPCHK(t, hipMemcpyAsync(b->d_in, img, len, hipMemcpyHostToDevice, t->stream));
    HIPCHK(t, hipStreamSynchronize(t->stream));
    return TCPEDIT_OK;
fail:
    return TCPEDIT_ERROR;
}

/* window mode's conditions: the wave lane's size-preserving instances over a native-order
 * microsecond image without a tcpprep cache (the window mode has no record numbers) */
static int fused_capable(const tcpedit_t *t, const tcpedit_batch_t *b)
{
    return b->fast_tiles && b->fast_kind == TE_FAST_WAVE && !b->slot_layout && static_capable(&t->cfg) &&
           fast_capable(&t->cfg) && !b->has_trim &&
           !b->swapped && !b->nsec && !b->d_dirbits && !b->pre_host && !fast_lane_off() &&
           b->stop_error_pkt < 0 && !b->walk_stop && b->n_pkts && !getenv("TCPEDIT_HIP_NO_FUSED");
}

static int win_ready(tcpedit_t *t, tcpedit_batch_t *b, uint64_t nwin)
{
    nwin = (nwin + 1) & ~1ull; /* (even: the verdict and chain-end words adjacent, one memset) */
    if (b->win_cap >= nwin)
        return 0;
    hipFree(b->d_win);
    b->d_win = NULL;
    b->win_cap = 0;
    if (hipMalloc((void **)&b->d_win, WIN_WS_BYTES(nwin)) != hipSuccess) {
        te_seterr(t, "out of device memory (window workspace)");
        return -1;
    }
    b->win_cap = nwin;
    return 0;
}

/* the window request over the batch's whole image */
static void win_request(const tcpedit_batch_t *b, te_win_req_t *q)
{
    memset(q, 0, sizeof(*q));
    q->len = b->in_len;
    q->entry = b->rec0 ? b->rec0 : 24;
    q->base = q->entry & ~15ull;
    q->limit = b->walk_limit ? b->walk_limit : b->in_len;
    q->nwin = (uint32_t)((q->limit - q->base + te_win_bytes() - 1) / te_win_bytes());
}

/* one window-mode run, results read back; 1 when the exact path has to run instead */
static int fused_once(tcpedit_t *t, tcpedit_batch_t *b)
{
    te_win_req_t q;
    win_request(b, &q);
    if (q.nwin == 0 || win_ready(t, b, q.nwin) < 0)
        return 1;
    out_header(t, b->ohdr);
    HIPCHK(t, hipMemcpyAsync(b->d_out, b->ohdr, 24, hipMemcpyHostToDevice, t->stream));
    HIPCHK(t, hipEventRecord(b->ev0, t->stream));
    b->win_req = &q;
    const int lr = launch(b, -1);
    b->win_req = NULL;
    if (lr != 0)
        return 1;
    HIPCHK(t, hipEventRecord(b->ev1, t->stream));
    uint32_t bad = 0;
    uint64_t tot = 0;
    const uint8_t *wb = b->d_win + WIN_BAD_OFF(b->win_cap);
    HIPCHK(t, hipMemcpyAsync(&bad, wb, 4, hipMemcpyDeviceToHost, t->stream));
    HIPCHK(t, hipMemcpyAsync(&tot, b->d_win + WIN_TOT_OFF(b->win_cap), 8, hipMemcpyDeviceToHost,
                             t->stream));
    if (!b->slots_host)
        b->slots_host = malloc(8 * TE_WK_SLOT_WORDS * (size_t)te_wave_grid());
    if (b->last_fgrid)
        HIPCHK(t, hipMemcpyAsync(b->slots_host, b->d_ws + WS_SLOTS(b->n_tiles),
                                 8 * TE_WK_SLOT_WORDS * (size_t)b->last_fgrid, hipMemcpyDeviceToHost, t->stream));
    HIPCHK(t, hipStreamSynchronize(t->stream));
    memset(b->counters, 0, sizeof(b->counters));
    for (int i = 0; i < b->last_fgrid; i++) {
        const uint64_t *v = b->slots_host + TE_WK_SLOT_WORDS * (size_t)i;
        b->counters[TE_CNT_PACKETS] += v[0];
        b->counters[TE_CNT_WRITTEN] += v[0];
        b->counters[TE_CNT_BYTES_IN] += v[1];
        b->counters[TE_CNT_BYTES_OUT] += v[1];
        b->counters[TE_CNT_EDITED] += v[2];
    }
    /* the chain ran where the host walk ran: to its end, every record (the index the batch
       was opened with counts them) */
    if (bad || tot != b->walk_end || b->counters[TE_CNT_PACKETS] != b->n_pkts || b->stop_error_pkt >= 0 ||
        b->walk_stop)
        return 1;
    float ms = 0;
    HIPCHK(t, hipEventElapsedTime(&ms, b->ev0, b->ev1));
    b->kernel_ms = ms;
    HIPCHK(t, hipMemsetAsync(b->d_status, 0, b->n_pkts ? b->n_pkts : 1, t->stream)); /* every record OK */
    HIPCHK(t, hipStreamSynchronize(t->stream));
    b->err[0] = b->err[1] = ~0ull;
    b->err[2] = 0;
    b->last_fast = 1;
    b->last_listed = 0;
    b->ran = 1;
    b->status_valid = 0;
    t->pub.runtime.packetnum += b->counters[TE_CNT_PACKETS];
    t->pub.runtime.total_bytes += b->counters[TE_CNT_BYTES_OUT];
    t->pub.runtime.pkts_edited += b->counters[TE_CNT_EDITED];
    return 0;
fail:
    return -1;
}

/* tcpedit_batch_run with the record discovery fused into the wave lane (window mode): no
 * index pass and no tiles -- each wave finds the records of its byte window itself, edits
 * them where they lie and the chain is checked across windows after.  Configs and images
 * the window mode does not carry, and any batch where a window misses the chain or leaves
 * a record to the generic lane, run the exact path (tcpedit_batch_run): the output is the
 * same either way. */
int tcpedit_batch_run_fused(tcpedit_t *t, tcpedit_batch_t *b)
{
    if (!t || !b)
        return TCPEDIT_ERROR;
    if (fused_capable(t, b)) {
        if (te_upload_cfg(t) < 0)
            return TCPEDIT_ERROR;
        const int r = fused_once(t, b);
        if (r == 0)
            return TCPEDIT_OK;
        if (r < 0)
            return TCPEDIT_ERROR;
        b->win_fallbacks++;
    }
    return tcpedit_batch_run(t, b);
}

/* K window-mode runs back to back (the device pipeline with the record discovery fused:
 * the wave lane + the chain check), hipEvents around them; TCPEDIT_ERROR when the batch is
 * not one the window mode carries */
int tcpedit_batch_time_fused(tcpedit_t *t, tcpedit_batch_t *b, int iters, double *ms_per_run)
{
    hipEvent_t e0 = NULL, e1 = NULL;
    float ms = 0;
    int rc = TCPEDIT_ERROR;
    if (!t || !b || iters <= 0 || !fused_capable(t, b) || te_upload_cfg(t) < 0)
        return TCPEDIT_ERROR;
    te_win_req_t q;
    win_request(b, &q);
    if (q.nwin == 0 || win_ready(t, b, q.nwin) < 0)
        return TCPEDIT_ERROR;
    HIPCHK(t, hipEventCreate(&e0));
    HIPCHK(t, hipEventCreate(&e1));
    HIPCHK(t, hipEventRecord(e0, t->stream));
    b->win_req = &q;
    for (int i = 0; i < iters; i++)
        if (launch(b, -1) != 0) {
            b->win_req = NULL;
            te_seterr(t, "kernel launch failed");
            goto fail;
        }
    b->win_req = NULL;
    HIPCHK(t, hipEventRecord(e1, t->stream));
    HIPCHK(t, hipEventSynchronize(e1));
    HIPCHK(t, hipEventElapsedTime(&ms, e0, e1));
    *ms_per_run = ms / iters;
    rc = TCPEDIT_OK;
fail:
    if (e0)
        hipEventDestroy(e0);
    if (e1)
        hipEventDestroy(e1);
    return rc;
}

uint64_t tcpedit_batch_fused_fallbacks(tcpedit_batch_t *b) { return b ? b->win_fallbacks : 0; }
uint64_t tcpedit_pipeline_fallbacks(tcpedit_t *t) { return t ? t->pipe_fallbacks : 0; }

int tcpedit_batch_run(tcpedit_t *t, tcpedit_batch_t *b)
{
    if (!t || !b)
        return TCPEDIT_ERROR;
    if (batch_run_dir(t, b, -1) != TCPEDIT_OK)
        return TCPEDIT_ERROR;
    if (b->counters[TE_CNT_Q8_FAILED]) {
        const uint8_t *st = tcpedit_batch_status(b);
        int64_t first = -1;
        for (uint64_t i = 0; st && i < b->n_pkts; i++)
            if (st[i] & TE_ST_UNSUPPORTED) {
                first = (int64_t)i;
                break;
            }
        te_seterr(t,
                  "record %lld: its edit reads the reference's stale static packet buffer (SURVEY Appendix B "
                  "Q8) at bytes the device replay cannot reconstruct (they come from before this batch, or "
                  "from bytes no record wrote)",
                  (long long)(first + 1 + (int64_t)b->pkt_base));
        return TCPEDIT_ERROR;
    }
    if (b->err[0] != ~0ull) {
        te_seterr(t, "Error rewriting packets: packet %lld", (long long)(b->err[0] + 1 + b->pkt_base));
        return TCPEDIT_ERROR;
    }
    if (b->stop_error_pkt >= 0) {
        te_seterr(t, TE_READER_ERR, (long long)(b->stop_error_pkt + 1 + (int64_t)b->pkt_base));
        return TCPEDIT_ERROR;
    }
    return TCPEDIT_OK;
}

int tcpedit_batch_result(tcpedit_batch_t *b, tcpedit_batch_result_t *r)
{
    if (!b || !r || !b->ran)
        return TCPEDIT_ERROR;
    memset(r, 0, sizeof(*r));
    r->packets = b->counters[TE_CNT_PACKETS];
    r->bytes_in = b->counters[TE_CNT_BYTES_IN];
    r->bytes_out = b->counters[TE_CNT_BYTES_OUT];
    r->written = b->counters[TE_CNT_WRITTEN];
    r->edited = b->counters[TE_CNT_EDITED];
    r->soft_errors = b->counters[TE_CNT_SOFT];
    r->warnings = b->counters[TE_CNT_WARN];
    r->errors = b->counters[TE_CNT_ERROR];
    r->unsupported = b->counters[TE_CNT_Q8_FAILED];
    r->stale_records = b->counters[TE_CNT_UNSUPPORTED];
    r->first_error = b->err[0] != ~0ull ? (int64_t)b->err[0] : -1;
    r->first_unsupported = -1;
    if (r->unsupported) {
        const uint8_t *st = tcpedit_batch_status(b);
        for (uint64_t i = 0; st && i < b->n_pkts; i++)
            if (st[i] & TE_ST_UNSUPPORTED) {
                r->first_unsupported = (int64_t)i;
                break;
            }
    }
    /* a hard error truncates the output at the failing record (tcprewrite.c:156-160) */
    uint64_t end = 24 + b->counters[TE_CNT_BYTES_OUT];
    if (b->err[0] != ~0ull)
        end = b->err[1];
    else if (b->stop_error_pkt >= 0)
        r->first_error = b->stop_error_pkt;
    r->out_len = end;
    r->n_tiles = (uint32_t)b->n_tiles;
    r->kernel_ms = b->kernel_ms;
    r->fast_lane = (uint32_t)b->last_fast;
    r->generic_tiles = b->last_fast ? b->last_listed : (uint32_t)b->n_tiles;
    r->fast_kind = b->last_fast ? (uint32_t)b->fast_kind : 0;
    return TCPEDIT_OK;
}

size_t tcpedit_batch_output(tcpedit_batch_t *b, void *dst, size_t cap)
{
    tcpedit_batch_result_t r;
    if (tcpedit_batch_result(b, &r) != TCPEDIT_OK)
        return 0;
    size_t n = r.out_len < cap ? r.out_len : cap;
    if (hipMemcpy(dst, b->d_out, n, hipMemcpyDeviceToHost) != hipSuccess)
        return 0;
    return n;
}

size_t tcpedit_batch_output_records(tcpedit_batch_t *b, void *dst, size_t cap)
{
    tcpedit_batch_result_t r;
    if (tcpedit_batch_result(b, &r) != TCPEDIT_OK || r.out_len < 24)
        return 0;
    size_t n = r.out_len - 24 < cap ? r.out_len - 24 : cap;
    if (n && hipMemcpy(dst, b->d_out + 24, n, hipMemcpyDeviceToHost) != hipSuccess)
        return 0;
    return n;
}

const void *tcpedit_batch_device_output(tcpedit_batch_t *b) { return b ? b->d_out : NULL; }

/* a direction array already on the device (te_replay.c: the --include/--exclude list as a
   tcpprep cache body), in place of the batch's; the batch owns d_bits from here on */
int te_batch_set_dirbits_dev(tcpedit_batch_t *b, uint8_t *d_bits, uint64_t len)
{
    if (!b)
        return -1;
    hipFree(b->d_dirbits);
    b->d_dirbits = d_bits;
    b->dirbits_len = len;
    b->status_valid = 0;
    return 0;
}
uint64_t tcpedit_batch_input_bytes(tcpedit_batch_t *b) { return b ? b->in_len : 0; }

/* The record index built on the device (te_index.hip) from the batch's device image,
 * replacing the host walk's: the count, scan and write passes `iters` times after one
 * sizing run; *ms = device ms per index build (HIP events).  Returns 0 applied, 1 not
 * served here (the config's tiles are not wave-lane tiles over contiguous records, or a
 * speculative guess missed the chain: the host index stays), -1 error. */
/* diagnostics / host tests (the sanitizer and thread-sanitizer runs): the host record
 * walk (index_image, the walker pool included) over a pcap image, without the device */
int tcpedit_debug_index_host(tcpedit_t *t, const void *pcap, size_t len, uint64_t *n_pkts, uint64_t *n_tiles,
                             uint64_t *walk_end)
{
    if (!t || !pcap)
        return TCPEDIT_ERROR;
    if (te_ensure_cfg(t) < 0)
        return TCPEDIT_ERROR;
    tcpedit_batch_t *b = calloc(1, sizeof(*b));
    if (!b)
        return TCPEDIT_ERROR;
    b->ctx = t;
    const int rc = index_image(t, b, (const uint8_t *)pcap, (const uint8_t *)pcap + (len >= 24 ? 24 : 0), len);
    if (rc == 0) {
        if (n_pkts)
            *n_pkts = b->n_pkts;
        if (n_tiles)
            *n_tiles = b->n_tiles;
        if (walk_end)
            *walk_end = b->walk_end;
    }
    free(b->tiles);
    free(b->pkt_rel);
    for (int i = 0; i < 64; i++) {
        free(b->wk_tiles[i]);
        free(b->wk_rel[i]);
    }
    free(b);
    return rc < 0 ? TCPEDIT_ERROR : TCPEDIT_OK;
}

static double te_now(void);
/* diagnostics / bench: the per-packet API's latency -- `iters` tcpedit_packet calls on
 * one packet as tcprewrite makes them (its buffer reused, tcprewrite.c:301-317), wall
 * microseconds per call */
int tcpedit_debug_packet_latency(tcpedit_t *t, const uint8_t *pkt, uint32_t caplen, int iters, double *us)
{
    if (!t || !pkt || iters < 1 || caplen > 262144u)
        return TCPEDIT_ERROR;
    unsigned char *buf = malloc(262144 + 4096);
    if (!buf)
        return TCPEDIT_ERROR;
    struct pcap_pkthdr h;
    int rc = TCPEDIT_OK;
    double t0 = 0;
    for (int i = -1; i < iters && rc != TCPEDIT_ERROR; i++) { /* (call -1: first-use staging, untimed) */
        if (i == 0)
            t0 = te_now();
        memset(&h, 0, sizeof h);
        h.caplen = h.len = caplen;
        memcpy(buf, pkt, caplen);
        struct pcap_pkthdr *hp = &h;
        unsigned char *d = buf;
        rc = tcpedit_packet(t, &hp, &d, TCPR_DIR_C2S);
    }
    if (us)
        *us = (te_now() - t0) * 1e6 / iters;
    free(buf);
    return rc == TCPEDIT_ERROR ? TCPEDIT_ERROR : TCPEDIT_OK;
}

/* the device index's workspace for a capture of `len` bytes from file offset `entry`:
 * the zeroed words and look-back granules, then the per-window records */
static uint64_t idx_nwin(uint64_t base, uint64_t limit)
{
    const uint64_t W = te_index_window_bytes();
    return limit > base ? (limit - base + W - 1) / W : 0;
}

static void idx_layout(IdxArgs *a, uint8_t *ws, uint64_t nwin)
{
    uint64_t *w = (uint64_t *)ws;
    a->totals = w;
    w += IDX_T__N + 2;
    a->w_entry = w;
    a->w_exit = w + nwin;
    a->w_agg = w + 2 * nwin;
    a->w_scr = w + 3 * nwin;
    a->w_pfx = w + 4 * nwin;
    a->w_sbase = w + 5 * nwin;
    a->w_prev = (int64_t *)(w + 6 * nwin);
    a->parts = w + 7 * nwin;
    a->t_tile = (uint32_t *)(w + 7 * nwin + IDX_PART_BYTES / 8 * (nwin / IDX_SB + 2));
    a->w_flags = a->t_tile + 2ull * IDX_MAXR * nwin;
    a->t_prel = (uint16_t *)(a->w_flags + nwin + 1);
}

int tcpedit_batch_index_device(tcpedit_t *t, tcpedit_batch_t *b, int iters, double *ms)
{
    if (!t || !b || iters < 1)
        return TCPEDIT_ERROR;
    if (!b->cut_device_ok || b->in_len <= 24)
        return 1;
    const uint64_t nwin = idx_nwin(16, b->in_len);
    if (nwin > 0x7fffffffull)
        return 1;
    uint8_t *wbuf = NULL;
    hipEvent_t e0 = NULL, e1 = NULL;
    int rc = TCPEDIT_ERROR;
    uint64_t tot[IDX_T__N];
    const uint64_t wsb = IDX_WS_BYTES(nwin);
    /* records and tiles: a tile never spans two windows, so at most one more a window */
    const uint64_t tile_cap = b->n_tiles + nwin + 1;
    te_tile_t *d_tiles = NULL;
    uint16_t *d_rel = NULL;
    HIPCHK(t, hipMalloc((void **)&wbuf, wsb));
    HIPCHK(t, hipMalloc((void **)&d_tiles, sizeof(te_tile_t) * tile_cap));
    HIPCHK(t, hipMalloc((void **)&d_rel, sizeof(uint16_t) * (b->n_pkts + 1)));
    IdxArgs a;
    memset(&a, 0, sizeof a);
    a.img = b->d_in;
    a.len = b->in_len;
    a.entry = 24;
    a.base = 16;
    a.limit = b->in_len;
    a.sw = b->swapped;
    a.nsec = b->nsec;
    a.nwin = (uint32_t)nwin;
    a.budget = b->cut_budget;
    a.max_pkts = b->cut_max_pkts;
    a.growth = b->cut_growth;
    idx_layout(&a, wbuf, nwin);
    a.tiles = d_tiles;
    a.pkt_rel = d_rel;
    a.tile_cap = tile_cap;
    a.rec_cap = b->n_pkts + 1;
    /* the index is built into its own tiles and record offsets, swapped in below (a
       missed guess leaves the host index as it is) */
    HIPCHK(t, hipEventCreate(&e0));
    HIPCHK(t, hipEventCreate(&e1));
    for (int i = -1; i < iters; i++) { /* (run -1: the check run, untimed) */
        if (i == 0)
            HIPCHK(t, hipEventRecord(e0, t->stream));
        if (te_launch_index(&a, t->stream)) {
            te_seterr(t, "device index launch failed: %s", hipGetErrorString(hipGetLastError()));
            goto out;
        }
        if (i == -1) {
            HIPCHK(t, hipMemcpyAsync(tot, a.totals, sizeof tot, hipMemcpyDeviceToHost, t->stream));
            HIPCHK(t, hipStreamSynchronize(t->stream));
            if (tot[IDX_T_BAD]) { /* a guess missed the chain: the host index stays (it is exact) */
                if (getenv("TCPEDIT_HIP_IDX_DEBUG")) {
                    const uint64_t q = tot[IDX_T_BADWIN];
                    uint64_t we[3] = {0, 0, 0}, wx[3] = {0, 0, 0};
                    uint32_t wf[3] = {0, 0, 0};
                    if (q != 0xffffffffull && q < nwin) {
                        const uint64_t q0 = q ? q - 1 : 0, n = q + 2 <= nwin ? q + 2 - q0 : nwin - q0;
                        hipMemcpy(we, a.w_entry + q0, 8 * n, hipMemcpyDeviceToHost);
                        hipMemcpy(wx, a.w_exit + q0, 8 * n, hipMemcpyDeviceToHost);
                        hipMemcpy(wf, a.w_flags + q0, 4 * n, hipMemcpyDeviceToHost);
                    }
                    fprintf(stderr, "device index: bad window %llu of %llu (timeouts? %llu); entry/exit/flags around it: "
                            "[%llx %llx %x] [%llx %llx %x] [%llx %llx %x]\n", (unsigned long long)q,
                            (unsigned long long)nwin, (unsigned long long)tot[IDX_T_WINDOWS],
                            (unsigned long long)we[0], (unsigned long long)wx[0], wf[0], (unsigned long long)we[1],
                            (unsigned long long)wx[1], wf[1], (unsigned long long)we[2], (unsigned long long)wx[2], wf[2]);
                }
                rc = 1;
                goto out;
            }
            if (tot[IDX_T_OVERFLOW] || tot[IDX_T_RECS] != b->n_pkts) { /* the chain is the chain */
                te_seterr(t, "device index found %llu records (overflow %llu), the host walk %llu",
                          (unsigned long long)tot[IDX_T_RECS], (unsigned long long)tot[IDX_T_OVERFLOW],
                          (unsigned long long)b->n_pkts);
                goto out;
            }
            if (tot[IDX_T_SCRATCH] > b->scratch_bytes) {
                hipFree(b->d_scratch);
                b->d_scratch = NULL;
                HIPCHK(t, hipMalloc((void **)&b->d_scratch, tot[IDX_T_SCRATCH]));
                b->scratch_bytes = tot[IDX_T_SCRATCH];
            }
        }
    }
    HIPCHK(t, hipEventRecord(e1, t->stream));
    HIPCHK(t, hipEventSynchronize(e1));
    {
        float f = 0;
        HIPCHK(t, hipEventElapsedTime(&f, e0, e1));
        if (ms)
            *ms = f / iters;
    }
    {
        const uint64_t nt = tot[IDX_T_TILES];
        if (nt > b->n_tiles) { /* tiles never span windows: there may be a few more */
            hipFree(b->d_tile_list);
            b->d_tile_list = NULL;
            hipFree(b->d_ws);
            b->d_ws = NULL;
            HIPCHK(t, hipMalloc((void **)&b->d_tile_list, sizeof(uint32_t) * (nt + 1)));
            b->ws_bytes = WS_SLOTS(nt) + 64 + (b->fast_kind == TE_FAST_WAVE ? 8 * TE_WK_SLOT_WORDS * (uint64_t)te_wave_grid() : 0);
            HIPCHK(t, hipMalloc((void **)&b->d_ws, b->ws_bytes));
        }
        hipFree(b->d_tiles);
        b->d_tiles = d_tiles;
        b->tcut_ok = 0;
        d_tiles = NULL;
        hipFree(b->d_pkt_rel);
        b->d_pkt_rel = d_rel;
        d_rel = NULL;
        b->n_tiles = nt;
    }
    b->has_trim = tot[IDX_T_TRIM] != 0;
    b->walk_end = tot[IDX_T_END];
    b->walk_stop = tot[IDX_T_STOP] == IDX_STOP ? 1 : tot[IDX_T_STOP] == IDX_ERROR ? 2 : 0;
    b->stop_error_pkt = tot[IDX_T_ERR_REC] == ~0ull ? -1 : (int64_t)tot[IDX_T_ERR_REC];
    b->out_cap = 24 + 64 + tot[IDX_T_BYTES];
    /* the lane hints and the wave lane's per-block slots follow the new tiles */
    HIPCHK(t, hipMemsetAsync(b->d_ws, 0, b->ws_bytes, t->stream));
    HIPCHK(t, hipStreamSynchronize(t->stream));
    b->gen_hint_ok = 0;
    b->launches = 0;
    b->last_listed = 0;
    b->status_valid = 0;
    rc = 0;
out:
    if (e0)
        hipEventDestroy(e0);
    if (e1)
        hipEventDestroy(e1);
    hipFree(d_tiles);
    hipFree(d_rel);
    hipFree(wbuf);
    return rc;
fail:
    rc = TCPEDIT_ERROR;
    goto out;
}

int tcpedit_batch_time(tcpedit_t *t, tcpedit_batch_t *b, int iters, double *ms_per_run)
{
    hipEvent_t e0, e1;
    float ms = 0;
    if (!t || !b || iters <= 0 || te_upload_cfg(t) < 0)
        return TCPEDIT_ERROR;
    HIPCHK(t, hipEventCreate(&e0));
    HIPCHK(t, hipEventCreate(&e1));
    HIPCHK(t, hipEventRecord(e0, t->stream));
    for (int i = 0; i < iters; i++)
        if (launch(b, -1) != 0) {
            te_seterr(t, "kernel launch failed");
            return TCPEDIT_ERROR;
        }
    HIPCHK(t, hipEventRecord(e1, t->stream));
    HIPCHK(t, hipEventSynchronize(e1));
    HIPCHK(t, hipEventElapsedTime(&ms, e0, e1));
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    *ms_per_run = ms / iters;
    return TCPEDIT_OK;
fail:
    return TCPEDIT_ERROR;
}

int tcpedit_batch_time_kernels(tcpedit_t *t, tcpedit_batch_t *b, int iters, double *ms_per_run, double *ms_kernel)
{
    hipEvent_t e0 = NULL, e1 = NULL;
    float ms = 0;
    int rc = TCPEDIT_ERROR;
    if (!t || !b || iters <= 0 || te_upload_cfg(t) < 0)
        return TCPEDIT_ERROR;
    if (b->kev_n < 2 * iters) { /* grow the pool (kept for later calls: no creation in timed runs) */
        hipEvent_t *k = realloc(b->kev, sizeof(hipEvent_t) * 2 * (size_t)iters);
        if (!k)
            return TCPEDIT_ERROR;
        b->kev = k;
        while (b->kev_n < 2 * iters) {
            HIPCHK(t, hipEventCreate(&b->kev[b->kev_n]));
            b->kev_n++;
        }
    }
    HIPCHK(t, hipEventCreate(&e0));
    HIPCHK(t, hipEventCreate(&e1));
    HIPCHK(t, hipEventRecord(e0, t->stream));
    for (int i = 0; i < iters; i++)
        if (launch_ev(b, -1, b->kev[2 * i], b->kev[2 * i + 1], 0) != 0) {
            te_seterr(t, "kernel launch failed");
            goto fail;
        }
    HIPCHK(t, hipEventRecord(e1, t->stream));
    HIPCHK(t, hipEventSynchronize(e1));
    HIPCHK(t, hipEventElapsedTime(&ms, e0, e1));
    *ms_per_run = ms / iters;
    double ksum = 0;
    for (int i = 0; i < iters; i++) {
        float k = 0;
        HIPCHK(t, hipEventElapsedTime(&k, b->kev[2 * i], b->kev[2 * i + 1]));
        ksum += k;
    }
    *ms_kernel = ksum / iters;
    rc = TCPEDIT_OK;
fail:
    if (e0)
        hipEventDestroy(e0);
    if (e1)
        hipEventDestroy(e1);
    return rc;
}

int tcpedit_rewrite_pcap(tcpedit_t *t, const void *in, size_t in_len, const void *cache, size_t cache_len, void **out,
                         size_t *out_len)
{
    *out = NULL;
    *out_len = 0;
    tcpedit_batch_t *b = tcpedit_batch_open(t, in, in_len, cache, cache_len, 0);
    if (!b)
        return TCPEDIT_ERROR;
    int rc = tcpedit_batch_run(t, b);
    tcpedit_batch_result_t r;
    if (tcpedit_batch_result(b, &r) == TCPEDIT_OK && !r.unsupported) {
        *out = malloc(r.out_len ? r.out_len : 1);
        *out_len = tcpedit_batch_output(b, *out, r.out_len);
    }
    tcpedit_batch_close(b);
    return rc;
}

/* ------------------------------------------------------------------------- */
/* pipelined whole-image rewrite                      */
/*                                                                           */
/* The image is cut into chunks of whole records (the record walk stops at a */
/* byte budget).  Two device slots and three streams: while chunk k is       */
/* edited, chunk k+1 crosses PCIe towards the device and chunk k-1 back.     */
/* The caller's buffers are page-locked for the call (hipHostRegister), so   */
/* both copies are DMA from and to them directly.                            */
/* ------------------------------------------------------------------------- */
#include <time.h>
static double te_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* page-locked host memory for callers that read a capture straight into it: the
 * pipelined rewrite then skips hipHostRegister for that buffer */
/* (hipHostMalloc puts the pages on the device's NUMA node; pages on the other node, or
   malloc'd and hipHostRegister'ed, or the non-coherent and coherent flags measured the same
   on MI355X boxes: profiles/r05_e2e_ab.txt) */
void *tcpedit_host_alloc(size_t bytes)
{
    void *p = NULL;
    return hipHostMalloc(&p, bytes ? bytes : 1, 0) == hipSuccess ? p : NULL;
}
void tcpedit_host_free(void *p)
{
    if (p)
        hipHostFree(p);
}

/* is [p, p+n) already page-locked (hipHostMalloc'd or registered)? */
static int host_locked(const void *p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return a.type == hipMemoryTypeHost;
}

/* device slots a pipelined run rotates through: chunk k is finished (results read, a
   stale-buffer replay retried with the earlier chunks as prefix) while chunk k + 1 is
   indexed and edited and chunk k + 2 uploads -- into a third slot, so chunk k's input and
   index stand until it is finished.  The edit of chunk k writes its slot's output buffer
   once chunk k - SLOTS's download has left it: with three slots the last chunks' edits
   waited on downloads three chunks back (the download stream trails the uploads), so there
   are more (TE_PIPE_SLOTS_N overrides, A/B) */
#ifndef TE_PIPE_SLOTS_N
#define TE_PIPE_SLOTS_N 6
#endif
#define TE_PIPE_SLOTS TE_PIPE_SLOTS_N
#define TE_PIPE_ANCHORS 64 /* chunk starts kept (chunks are >= 8 MiB: >= 512 MiB of anchors) */
/* the default chunk: a tenth of the capture, 8-32 MiB (measured on MI355X, tools/e2e_probe.py:
   C2's 80 MB runs best at 8 MiB -- pipeline fill and drain are one chunk each -- and 2M IMIX
   records (740 MB) at 12-32 MiB, where per-chunk costs dominate) */
#define TE_PIPE_CHUNK_MIN ((size_t)8 << 20)
#define TE_PIPE_CHUNK_MAX ((size_t)32 << 20)

/* res_pinned layout: the workspace head (error words, ticket, both counter sets: one copy
   of d_ws[0, WS_STATE)) | wave-lane slots */
#define TE_RES_SLOTS WS_STATE
_Static_assert(WS_COUNTERS1 + 8 * TE_CNT__N <= WS_STATE && WS_ERR + 24 <= WS_COUNTERS, "workspace head layout");

/* the device-index pipeline uploads each chunk with the bytes of a record that starts in it
   and ends past it: the largest record (16 + 262144 bytes), rounded */
#define TE_PIPE_MARGIN ((size_t)262160 + 240)

struct te_pipe_s {
    size_t chunk;                      /* record-byte budget of a chunk (slot capacity) */
    hipStream_t s_h2d, s_d2h;
    tcpedit_batch_t *slot[TE_PIPE_SLOTS];
    hipEvent_t h2d_done[TE_PIPE_SLOTS], edit_done[TE_PIPE_SLOTS], d2h_done[TE_PIPE_SLOTS];
    uint64_t d_out_alloc[TE_PIPE_SLOTS], d_scratch_alloc[TE_PIPE_SLOTS];
    uint8_t *hdr;                      /* pinned copy of the 24-byte file header */
    /* the device record index (te_index.hip) per slot: its workspace, totals (pinned), done */
    uint8_t *d_idx[TE_PIPE_SLOTS];
    uint64_t *h_tot[TE_PIPE_SLOTS];
    hipEvent_t idx_done[TE_PIPE_SLOTS];
    uint64_t idx_nwin;
    /* the call's host image, and per slot the file offsets of its chunk's first record and
       of the previous chunk's (~0: none, the chunk is the capture's first) -- for the Q8
       replay's prefix records */
    const uint8_t *img;
    uint64_t first_off[TE_PIPE_SLOTS], prev_off[TE_PIPE_SLOTS];
    /* the latest chunks' first-record offsets (a ring): known record boundaries a Q8
       replay's prefix walk can start from instead of the capture's first record */
    uint64_t anchor[TE_PIPE_ANCHORS];
    uint32_t nanchor;
    /* per slot: the chunk's output already on its way down (its D2H issued right after the
       edit launch, a size-preserving config: output bytes = record bytes, known from the
       index totals), ~0 when not */
    uint64_t early[TE_PIPE_SLOTS];
    uint32_t early_miss, early_n; /* (trace: early copies done again, early copies) */
    /* the window-mode pipeline: the call's device accumulator {packets, bytes, edited,
       chain verdict} and its pinned landing area (+ the last chunk's chain end) */
    uint64_t *d_wacc, *h_wacc;
    /* slots opened so far: a call opens only as many as its capture can have chunks in
       flight (pipe_ready), later calls open more -- each slot is ~7x its chunk bytes of
       device memory (input, output, huge-record scratch, per-record index arrays: ~230 MB
       at a 32 MiB chunk) and its index arrays ~2x the chunk in page-locked host memory */
    int nopen;
};

/* a chunk's first record at file offset off: an anchor for later prefixes */
static void pipe_anchor(te_pipe_t *P, uint64_t off)
{
    if (P->nanchor && P->anchor[(P->nanchor - 1) % TE_PIPE_ANCHORS] >= off)
        return;
    P->anchor[P->nanchor++ % TE_PIPE_ANCHORS] = off;
}

/* where the prefix of the chunk starting at `first` may start: the newest anchor far enough
   back that the staged records (at most TE_Q8_PRE_BYTES, stage_prefix) are the same as a
   walk from the capture's start would stage, else the capture's first record (24) */
static uint64_t pipe_prefix_from(const te_pipe_t *P, uint64_t first)
{
    const uint64_t need = (uint64_t)TE_Q8_PRE_BYTES + 262144u + 16u;
    if (first < 24 + need)
        return 24;
    const uint32_t n = P->nanchor < TE_PIPE_ANCHORS ? P->nanchor : TE_PIPE_ANCHORS;
    uint64_t best = 24;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t a = P->anchor[(P->nanchor - 1 - i) % TE_PIPE_ANCHORS];
        if (a <= first - need) {
            best = a;
            break;
        }
    }
    return best;
}

void te_pipe_free(tcpedit_t *t)
{
    te_pipe_t *P = t->pipe;
    if (!P)
        return;
    for (int s = 0; s < TE_PIPE_SLOTS; s++) {
        if (P->slot[s]) {
            P->slot[s]->d_dirbits = NULL; /* the call's, freed there */
            tcpedit_batch_close(P->slot[s]);
        }
        if (P->h2d_done[s])
            hipEventDestroy(P->h2d_done[s]);
        if (P->edit_done[s])
            hipEventDestroy(P->edit_done[s]);
        if (P->d2h_done[s])
            hipEventDestroy(P->d2h_done[s]);
        if (P->idx_done[s])
            hipEventDestroy(P->idx_done[s]);
        hipFree(P->d_idx[s]);
        hipHostFree(P->h_tot[s]);
    }
    hipFree(P->d_wacc);
    hipHostFree(P->h_wacc);
    if (P->s_h2d)
        hipStreamDestroy(P->s_h2d);
    if (P->s_d2h)
        hipStreamDestroy(P->s_d2h);
    hipHostFree(P->hdr);
    free(P);
    t->pipe = NULL;
}

/* one device slot sized for `chunk` record bytes; index arrays pinned */
static tcpedit_batch_t *pipe_slot_open(tcpedit_t *t, size_t chunk)
{
    tcpedit_batch_t *b = calloc(1, sizeof(*b));
    b->ctx = t;
    b->idx_pinned = 1;
    b->grow_never = 1;
    /* a record is at least its 16-byte header; the device index may also take the records
       of a chunk's margin (TE_PIPE_MARGIN), and cut a tile more a window */
    b->idx_cap_pkts = (chunk + TE_PIPE_MARGIN) / 16 + 2;
    b->idx_cap_tiles = b->idx_cap_pkts + (chunk + TE_PIPE_MARGIN) / te_index_window_bytes() + 2;
    HIPCHK(t, hipHostMalloc((void **)&b->tiles, sizeof(te_tile_t) * b->idx_cap_tiles, 0));
    HIPCHK(t, hipHostMalloc((void **)&b->pkt_rel, sizeof(uint16_t) * b->idx_cap_pkts, 0));
    HIPCHK(t, hipMalloc((void **)&b->d_in, chunk + TE_PIPE_MARGIN + 24 + 64));
    HIPCHK(t, hipMalloc((void **)&b->d_status, b->idx_cap_pkts + 16));
    HIPCHK(t, hipMalloc((void **)&b->d_tiles, sizeof(te_tile_t) * (b->idx_cap_tiles + 1)));
    HIPCHK(t, hipMalloc((void **)&b->d_pkt_rel, sizeof(uint16_t) * (b->idx_cap_pkts + 1)));
    HIPCHK(t, hipMalloc((void **)&b->d_tile_list, sizeof(uint32_t) * (b->idx_cap_tiles + 1)));
    b->q8_cap = (uint32_t)(b->idx_cap_pkts < TE_Q8_CAP ? b->idx_cap_pkts : TE_Q8_CAP);
    HIPCHK(t, hipMalloc((void **)&b->d_q8, 16 * (size_t)b->q8_cap));
    HIPCHK(t, hipMalloc((void **)&b->d_ws, WS_SLOTS(b->idx_cap_tiles) + 64 + 8 * TE_WK_SLOT_WORDS * (uint64_t)te_wave_grid()));
    HIPCHK(t, hipHostMalloc((void **)&b->res_pinned, TE_RES_SLOTS + 8 * TE_WK_SLOT_WORDS * (uint64_t)te_wave_grid(), 0));
    HIPCHK(t, hipEventCreate(&b->ev0));
    HIPCHK(t, hipEventCreate(&b->ev1));
    return b;
fail:
    tcpedit_batch_close(b);
    return NULL;
}

/* the pipeline for `chunk`-byte chunks with at least `want` slots open (the chunks a capture
   of in_len bytes can be cut into, at most TE_PIPE_SLOTS: pipe_want) */
static int pipe_ready(tcpedit_t *t, size_t chunk, int want)
{
    te_pipe_t *P = t->pipe;
    if (want > TE_PIPE_SLOTS)
        want = TE_PIPE_SLOTS;
    if (want < 1)
        want = 1;
    if (P && P->chunk == chunk && P->nopen >= want)
        return 0;
    if (!P || P->chunk != chunk) {
        te_pipe_free(t);
        P = t->pipe = calloc(1, sizeof(*P));
        if (!P) {
            te_seterr(t, "out of memory");
            return -1;
        }
        for (int j = 0; j < TE_PIPE_SLOTS; j++)
            P->early[j] = ~0ull;
        P->chunk = chunk;
        HIPCHK(t, hipStreamCreateWithFlags(&P->s_h2d, hipStreamNonBlocking));
        HIPCHK(t, hipStreamCreateWithFlags(&P->s_d2h, hipStreamNonBlocking));
        HIPCHK(t, hipHostMalloc((void **)&P->hdr, 64, 0));
        P->idx_nwin = idx_nwin(16, 24 + chunk + TE_PIPE_MARGIN);
    }
    for (int s = P->nopen; s < want; s++, P->nopen++) {
        if (!(P->slot[s] = pipe_slot_open(t, chunk)))
            goto fail;
        HIPCHK(t, hipEventCreateWithFlags(&P->h2d_done[s], hipEventDisableTiming));
        HIPCHK(t, hipEventCreateWithFlags(&P->edit_done[s], hipEventDisableTiming));
        HIPCHK(t, hipEventCreateWithFlags(&P->d2h_done[s], hipEventDisableTiming));
        HIPCHK(t, hipEventCreateWithFlags(&P->idx_done[s], hipEventDisableTiming));
        HIPCHK(t, hipMalloc((void **)&P->d_idx[s], IDX_WS_BYTES(P->idx_nwin)));
        HIPCHK(t, hipHostMalloc((void **)&P->h_tot[s], 8 * IDX_T__N, 0));
    }
    return 0;
fail:
    te_pipe_free(t);
    return -1;
}

/* grow a slot's output / scratch buffers for a chunk that needs more (fixlen pad, huge records) */
static int pipe_grow(tcpedit_t *t, te_pipe_t *P, int s)
{
    tcpedit_batch_t *b = P->slot[s];
    if (b->out_cap + 64 > P->d_out_alloc[s] || b->scratch_bytes > P->d_scratch_alloc[s]) {
        HIPCHK(t, hipEventSynchronize(P->d2h_done[s]));
        HIPCHK(t, hipStreamSynchronize(t->stream));
    }
    if (b->out_cap + 64 > P->d_out_alloc[s]) {
        hipFree(b->d_out);
        b->d_out = NULL;
        P->d_out_alloc[s] = (b->out_cap + 64) + (b->out_cap + 64) / 4;
        HIPCHK(t, hipMalloc((void **)&b->d_out, P->d_out_alloc[s]));
    }
    if (b->scratch_bytes > P->d_scratch_alloc[s]) {
        hipFree(b->d_scratch);
        b->d_scratch = NULL;
        P->d_scratch_alloc[s] = b->scratch_bytes + b->scratch_bytes / 4;
        HIPCHK(t, hipMalloc((void **)&b->d_scratch, P->d_scratch_alloc[s]));
    }
    return 0;
fail:
    return -1;
}

/* a chunk's results are on the host: add the wave lane's block totals, check for
 * errors, and issue the D2H of its output records to *pos (chunks finish in order).
 * *stopped = 2 after a hard error: the output ends there and later chunks are dropped */
static int pipe_finish_chunk(tcpedit_t *t, te_pipe_t *P, int s, uint64_t pkt_base, uint8_t *dst, size_t out_cap,
                             uint64_t *pos, int *stopped)
{
    tcpedit_batch_t *b = P->slot[s];
    if (*stopped == 2)
        return 0;
    memcpy(b->counters, b->res_pinned + b->last_cnt_off, sizeof(b->counters));
    int retried = 0; /* a replay rewrote output bytes after the chunk's early D2H */
    if (b->counters[TE_CNT_Q8_FAILED] && P->img && P->prev_off[s] != ~0ull) {
        retried = 1;
        /* the stale bytes may come from earlier chunks: the replay walks back into their
           records (the host image holds them all; the staging keeps the newest) */
        /* from a chunk start about TE_Q8_PRE_BYTES back (the walk is O(bytes walked)); from
           the capture's first record only when the replay needs the buffer's initial zeros */
        const uint64_t from = pipe_prefix_from(P, P->first_off[s]);
        tcpedit_batch_set_prefix(t, b, P->img + from, P->first_off[s] - from);
        const uint64_t before = b->counters[TE_CNT_Q8_FAILED];
        int r = retry_q8_with_prefix(t, b, -1, b->counters);
        if (r == 0 && from != 24 && b->counters[TE_CNT_Q8_FAILED]) {
            tcpedit_batch_set_prefix(t, b, P->img + 24, P->first_off[s] - 24);
            r = retry_q8_with_prefix(t, b, -1, b->counters);
        }
        if (getenv("TCPEDIT_HIP_Q8_DEBUG"))
            fprintf(stderr, "q8 retry: slot %d first_off %llu pkt_base %llu failed %llu -> %llu (listed %llu) npre %u "
                    "file_start %d rc %d\n", s, (unsigned long long)P->first_off[s], (unsigned long long)b->pkt_base,
                    (unsigned long long)before, (unsigned long long)b->counters[TE_CNT_Q8_FAILED],
                    (unsigned long long)b->counters[TE_CNT_UNSUPPORTED], b->npre, b->pre_file_start, r);
        tcpedit_batch_set_prefix(t, b, NULL, 0);
        if (r < 0)
            return -1;
    }
    memcpy(b->err, b->res_pinned + WS_ERR, sizeof(b->err));
    for (int i = 0; i < b->last_fgrid; i++) {
        const uint64_t *v = (const uint64_t *)(b->res_pinned + TE_RES_SLOTS) + TE_WK_SLOT_WORDS * (size_t)i;
        b->counters[TE_CNT_PACKETS] += v[0];
        b->counters[TE_CNT_WRITTEN] += v[0];
        b->counters[TE_CNT_BYTES_IN] += v[1];
        b->counters[TE_CNT_BYTES_OUT] += v[1];
        b->counters[TE_CNT_EDITED] += v[2];
    }
    b->err[0] = ~b->err[0]; /* stored complemented (0 = no error -> ~0) */
    b->err[1] = ~b->err[1];
    if (b->err[2]) {
        te_seterr(t, "device look-back timed out (%llu tiles)", (unsigned long long)b->err[2]);
        return -1;
    }
    if (b->counters[TE_CNT_Q8_FAILED]) {
        te_seterr(t, "a record's edit reads the reference's stale static packet buffer (SURVEY Appendix B Q8) "
                     "at bytes written before the previous pipeline chunk or by no record: not reproducible here");
        return -1;
    }
    const uint64_t ob = b->out_base ? b->out_base : 24;
    uint64_t bytes = b->counters[TE_CNT_BYTES_OUT];
    int64_t err_pkt = -1;
    int reader_err = 0;
    if (b->err[0] != ~0ull) { /* a hard error truncates the output at the failing record */
        bytes = b->err[1] - ob;
        err_pkt = (int64_t)(pkt_base + b->err[0]);
    } else if (b->stop_error_pkt >= 0) {
        err_pkt = (int64_t)(pkt_base + (uint64_t)b->stop_error_pkt);
        reader_err = 1;
    }
    if (*pos + bytes > out_cap) {
        te_seterr(t, "output buffer too small (%llu bytes needed so far)", (unsigned long long)(*pos + bytes));
        return -1;
    }
    if (P->early[s] != ~0ull && (retried || P->early[s] != *pos))
        P->early_miss++;
    if (P->early[s] == ~0ull || retried || P->early[s] != *pos) {
        /* (an early copy landed where these bytes go, unless a replay changed them since;
           after a hard error it copied more than `bytes`, past the output's end) */
        HIPCHK(t, hipStreamWaitEvent(P->s_d2h, P->edit_done[s], 0));
        if (bytes)
            HIPCHK(t, hipMemcpyAsync(dst + *pos, b->d_out + ob, bytes, hipMemcpyDeviceToHost, P->s_d2h));
        HIPCHK(t, hipEventRecord(P->d2h_done[s], P->s_d2h));
    }
    P->early[s] = ~0ull;
    *pos += bytes;
    t->pub.runtime.packetnum += b->counters[TE_CNT_PACKETS];
    t->pub.runtime.total_bytes += b->counters[TE_CNT_BYTES_OUT];
    t->pub.runtime.pkts_edited += b->counters[TE_CNT_EDITED];
    if (err_pkt >= 0) {
        te_seterr(t, reader_err ? TE_READER_ERR : "Error rewriting packets: packet %lld", (long long)(err_pkt + 1));
        t->pipe_err = 1;
        *stopped = 2;
    }
    return 0;
fail:
    return -1;
}

size_t tcpedit_output_bound(tcpedit_t *t, const void *in, size_t in_len)
{
    const uint8_t *img = in;
    if (!t || !img || in_len < 24)
        return 0;
    if (te_is_pcapng(img, in_len)) { /* the classic image the reader delivers */
        uint8_t *ng = NULL;
        size_t ng_len = 0;
        if (te_pcapng_to_pcap(img, in_len, &ng, &ng_len, NULL, 0) < 0)
            return 24 + 64;
        const size_t b = tcpedit_output_bound(t, ng, ng_len);
        free(ng);
        return b;
    }
    uint32_t magic;
    memcpy(&magic, img, 4);
    const int sw = magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u;
    const int pad = t->cfg.fixlen == TE_FIXLEN_PAD;
    const size_t growth = rec_growth(&t->cfg);
    size_t bound = 24 + 64, off = 24, pf = 24;
    while (off + 16 <= in_len) {
        for (const size_t pf_end = off + 4096 < in_len ? off + 4096 : in_len; pf < pf_end; pf += 64)
            __builtin_prefetch(img + pf); /* see index_image */
        const uint32_t caplen = rd32(img + off + 8, sw), plen = rd32(img + off + 12, sw);
        if (caplen > 262144u || off + 16 + caplen > in_len)
            break;
        bound += 16 + (size_t)(pad && plen > caplen && plen <= 262144u ? plen : caplen) + growth;
        off += 16 + caplen;
    }
    return bound;
}

/* The chunk schedule of a device-index pipeline: file offsets of the chunks' first bytes,
 * st[0] = 24 ... st[n] = in_len.  The first and last chunks ramp (C/8, C/4, C/2 -- at least
 * 1 MiB, which holds any record), the rest are about C: the D2H stream starts after a
 * small first chunk is in and edited, and only a small last chunk's edit and D2H are left
 * when the last H2D ends (the run's fill and drain).  Every chunk but the last is a
 * multiple of 16 bytes long (the chunks' images share one 16-byte phase).  NULL: no memory. */
static uint64_t *pipe_plan(size_t in_len, size_t C, int *n_out)
{
    const uint64_t N = in_len > 24 ? in_len - 24 : 0, MIN = (uint64_t)1 << 20;
    uint64_t ramp[3];
    int nr = 0;
    for (int q = 3; q >= 1; q--) {
        const uint64_t r = ((C >> q) < MIN ? MIN : (uint64_t)(C >> q)) & ~15ull;
        if (r < C && (nr == 0 || ramp[nr - 1] != r))
            ramp[nr++] = r;
    }
    uint64_t ramp_sum = 0;
    for (int i = 0; i < nr; i++)
        ramp_sum += ramp[i];
    const int cap = (int)(N / MIN) + 2 * nr + 4;
    uint64_t *st = malloc(sizeof(uint64_t) * (size_t)cap);
    if (!st)
        return NULL;
    int n = 0;
    uint64_t at = 24;
    st[n++] = at;
    if (N > 2 * ramp_sum + C) {
        for (int i = 0; i < nr; i++)
            st[n++] = (at += ramp[i]);
        const uint64_t mid = N - 2 * ramp_sum, m = (mid + C - 1) / C, each = ((mid + m - 1) / m + 15) & ~15ull;
        for (uint64_t i = 0; i + 1 < m; i++)
            st[n++] = (at += each);
        st[n++] = (at = 24 + N - ramp_sum); /* (the middle's last chunk takes the remainder) */
        for (int i = nr - 1; i > 0; i--)
            st[n++] = (at += ramp[i]);
        st[n++] = in_len;
    } else { /* a small capture: pieces of at most C/2 (at least 1 MiB) */
        const uint64_t half = ((C / 2 < MIN ? MIN : C / 2) + 15) & ~15ull;
        while (in_len - at > half)
            st[n++] = (at += half);
        st[n++] = in_len;
    }
    /* (a chunk boundary past the end cannot happen: every step stays below in_len) */
    *n_out = n - 1;
    return st;
}

/* TCPEDIT_HIP_PIPE_INDEX=host keeps the host record walk in the pipeline (A/B) */
static int pipe_index_host_env(void)
{
    const char *e = getenv("TCPEDIT_HIP_PIPE_INDEX");
    return e && strcmp(e, "host") == 0;
}

/* The pipeline with the record index built on the device (te_index.hip), for the wave
 * lane's configs: chunk k is the file bytes [24 + kC, 24 + (k+1)C), uploaded with the next
 * TE_PIPE_MARGIN bytes (a record starting in it may end past it) -- a fixed byte range, so
 * its H2D never waits for the record walk.  Its records are the ones starting in the chunk
 * from where the previous chunk's chain ended; the device reads that position from the
 * previous chunk's index totals (same stream), so the host's only wait per chunk is for
 * the index's totals before it launches the edit.  A chunk whose speculation missed the
 * chain is walked on the host from the exact position instead (te_index.hip).
 * Returns 0 (*pos, the output end), or -1. */
static int pipe_run_dix(tcpedit_t *t, te_pipe_t *P, const uint8_t *img, size_t in_len, uint8_t *dst, size_t out_cap,
                        uint8_t *d_dirbits, uint64_t dirbits_len, uint64_t *pos_io, int trace)
{
    const size_t C = P->chunk;
    int nch = 0;
    /* equal chunks; TCPEDIT_HIP_PIPE_RAMP=1 ramps the first and last (A/B: on C2 it cost more
       in per-chunk overhead than it saved in fill and drain, 2.29 vs 2.15 ms) */
    uint64_t *cst = getenv("TCPEDIT_HIP_PIPE_RAMP") ? pipe_plan(in_len, C, &nch) : NULL;
    if (!cst) {
        nch = (int)((in_len - 24 + C - 1) / C);
        if (nch < 1)
            nch = 1;
        cst = malloc(sizeof(uint64_t) * ((size_t)nch + 1));
        if (!cst) {
            te_seterr(t, "out of memory");
            return -1;
        }
        for (int j = 0; j < nch; j++)
            cst[j] = 24 + (uint64_t)j * C;
        cst[nch] = in_len;
    }
    if (nch > P->nopen && P->nopen < TE_PIPE_SLOTS) { /* (pipe_ready's bound on the chunks) */
        te_seterr(t, "pipeline: %d chunks over %d open slots", nch, P->nopen);
        free(cst);
        return -1;
    }
    uint64_t pos = *pos_io, pkts = 0, chunk_pkt_base[TE_PIPE_SLOTS] = {0};
    int inflight[TE_PIPE_SLOTS] = {0}, stopped = 0, k = 0, fallbacks = 0;
    uint64_t entry_file = 24;  /* host copy of where chunk k's records start (file offset) */
    uint64_t prev_first = ~0ull;
    P->img = img;
    P->nanchor = 0; /* (this call's capture) */
    uint64_t limit_img[TE_PIPE_SLOTS] = {0}, file0[TE_PIPE_SLOTS] = {0};
    IdxArgs A[TE_PIPE_SLOTS];
    const double t0 = te_now();
    double t_wait = 0;
    /* chunk j: upload into its slot (the slot's previous edit must be done reading d_in) */
#define DIX_UPLOAD(j)                                                                                         \
    do {                                                                                                      \
        const int s_ = (j) % TE_PIPE_SLOTS;                                                                   \
        tcpedit_batch_t *b_ = P->slot[s_];                                                                    \
        const uint64_t f0_ = cst[j], f1_ = cst[(j) + 1];                                                     \
        const uint64_t fe_ = f1_ + TE_PIPE_MARGIN < in_len ? f1_ + TE_PIPE_MARGIN : in_len;                  \
        if ((j) >= TE_PIPE_SLOTS)                                                                             \
            HIPCHK(t, hipStreamWaitEvent(P->s_h2d, P->edit_done[s_], 0));                                     \
        HIPCHK(t, hipMemcpyAsync(b_->d_in, P->hdr, 24, hipMemcpyHostToDevice, P->s_h2d));                     \
        HIPCHK(t, hipMemcpyAsync(b_->d_in + 24, img + f0_, fe_ - f0_, hipMemcpyHostToDevice, P->s_h2d));      \
        HIPCHK(t, hipEventRecord(P->h2d_done[s_], P->s_h2d));                                                 \
        b_->in_len = 24 + (fe_ - f0_);                                                                        \
        file0[s_] = f0_;                                                                                      \
        limit_img[s_] = f1_ >= in_len ? b_->in_len : 24 + (f1_ - f0_);                                       \
    } while (0)
    /* chunk j's index on the compute stream, after its upload; its first record from the
       previous chunk's totals (on the device), or 24 */
#define DIX_INDEX(j)                                                                                          \
    do {                                                                                                      \
        const int s_ = (j) % TE_PIPE_SLOTS, ps_ = ((j) + TE_PIPE_SLOTS - 1) % TE_PIPE_SLOTS;                  \
        tcpedit_batch_t *b_ = P->slot[s_];                                                                    \
        IdxArgs *a_ = &A[s_];                                                                                 \
        memset(a_, 0, sizeof *a_);                                                                            \
        a_->img = b_->d_in;                                                                                   \
        a_->len = b_->in_len;                                                                                 \
        a_->entry = 24;                                                                                       \
        a_->entry_ptr = (j) ? A[ps_].totals + IDX_T_END : NULL;                                               \
        a_->entry_sub = (j) ? cst[j] - cst[(j) - 1] : 0; /* the previous chunk's image is that much earlier */ \
        a_->base = 16;                                                                                        \
        a_->limit = limit_img[s_];                                                                            \
        a_->sw = b_->swapped;                                                                                 \
        a_->nsec = b_->nsec;                                                                                  \
        a_->nwin = (uint32_t)idx_nwin(16, limit_img[s_]);                                                     \
        a_->budget = b_->cut_budget;                                                                          \
        a_->max_pkts = b_->cut_max_pkts;                                                                      \
        a_->growth = b_->cut_growth;                                                                          \
        idx_layout(a_, P->d_idx[s_], a_->nwin);                                                               \
        a_->tiles = b_->d_tiles;                                                                              \
        a_->pkt_rel = b_->d_pkt_rel;                                                                          \
        a_->tile_cap = b_->idx_cap_tiles;                                                                     \
        a_->rec_cap = b_->idx_cap_pkts;                                                                       \
        HIPCHK(t, hipStreamWaitEvent(t->stream, P->h2d_done[s_], 0));                                        \
        if (te_launch_index(a_, t->stream)) {                                                                 \
            te_seterr(t, "device index launch failed: %s", hipGetErrorString(hipGetLastError()));            \
            goto fail;                                                                                        \
        }                                                                                                     \
        HIPCHK(t, hipMemcpyAsync(P->h_tot[s_], a_->totals, 8 * IDX_T__N, hipMemcpyDeviceToHost, t->stream)); \
        HIPCHK(t, hipEventRecord(P->idx_done[s_], t->stream));                                                \
    } while (0)

    uint64_t pos_early = pos; /* where the next early D2H lands (size-preserving configs) */
    for (int j = 0; j < TE_PIPE_SLOTS; j++)
        P->early[j] = ~0ull;
    P->early_n = P->early_miss = 0;
    DIX_UPLOAD(0);
    DIX_INDEX(0);
    for (;; k++) {
        const int s = k % TE_PIPE_SLOTS;
        tcpedit_batch_t *b = P->slot[s];
        const int more = k + 1 < nch;
        if (more)
            DIX_UPLOAD(k + 1);
        /* ---- chunk k's index totals ---- */
        const double tw = te_now();
        HIPCHK(t, hipEventSynchronize(P->idx_done[s]));
        t_wait += te_now() - tw;
        const uint64_t *T = P->h_tot[s];
        const uint64_t entry_img = entry_file - file0[s] + 24, chunk_first = entry_file;
        b->pkt_base = pkts;
        b->launches = 0;
        b->gen_hint_ok = 0;
        free(b->slots_host);
        b->slots_host = NULL;
        /* the chunk's first record sits at entry_img (bytes before it end the previous
           chunk's last record); its output at an offset of the same 16-byte phase (the
           wave lane stores whole 16-byte chunks at input offsets + a multiple of 16) */
        b->rec0 = entry_img;
        b->out_base = 24 + ((entry_img - 24) & 15);
        if (T[IDX_T_BAD] || T[IDX_T_OVERFLOW] || T[IDX_T_RECS] > b->idx_cap_pkts) {
            /* the speculation missed the chain: walk this chunk on the host from the exact
               position, and give the next chunk's index that walk's end */
            fallbacks++;
            b->walk_from = entry_img;
            b->walk_limit = limit_img[s];
            const int rc = index_image(t, b, img, img + file0[s], b->in_len);
            b->walk_from = b->walk_limit = 0;
            if (rc < 0)
                goto fail;
            b->out_cap += 16; /* (out_base) */
            HIPCHK(t, hipMemcpyAsync(b->d_tiles, b->tiles, sizeof(te_tile_t) * b->n_tiles, hipMemcpyHostToDevice,
                                     t->stream));
            b->tcut_ok = 0;
            HIPCHK(t, hipMemcpyAsync(b->d_pkt_rel, b->pkt_rel, sizeof(uint16_t) * b->n_pkts, hipMemcpyHostToDevice,
                                     t->stream));
            P->h_tot[s][IDX_T_END] = b->walk_end;
            HIPCHK(t, hipMemcpyAsync(A[s].totals + IDX_T_END, &P->h_tot[s][IDX_T_END], 8, hipMemcpyHostToDevice,
                                     t->stream));
        } else {
            b->n_pkts = T[IDX_T_RECS];
            b->n_tiles = T[IDX_T_TILES];
            b->has_trim = T[IDX_T_TRIM] != 0;
            b->walk_end = T[IDX_T_END];
            b->walk_stop = T[IDX_T_STOP] == IDX_STOP ? 1 : T[IDX_T_STOP] == IDX_ERROR ? 2 : 0;
            b->stop_error_pkt = T[IDX_T_ERR_REC] == ~0ull ? -1 : (int64_t)T[IDX_T_ERR_REC];
            b->out_cap = 24 + 16 + 64 + T[IDX_T_BYTES];
            b->scratch_bytes = T[IDX_T_SCRATCH];
            if (T[IDX_T_SCRATCH] > P->d_scratch_alloc[s]) {
                te_seterr(t, "device index scratch %llu > %llu", (unsigned long long)T[IDX_T_SCRATCH],
                          (unsigned long long)P->d_scratch_alloc[s]);
                goto fail;
            }
        }
        entry_file = file0[s] + b->walk_end - 24;
        if (b->n_pkts == 0) {
            if (b->stop_error_pkt >= 0) { /* the chunk's first record is the hard error: the
                                             output ends with the chunks before (utils.c:136-156) */
                te_seterr(t, TE_READER_ERR, (long long)(pkts + 1));
                t->pipe_err = 1;
            }
            stopped = 1;
        } else {
            if (b->walk_stop || b->walk_end + 16 > b->in_len)
                stopped = 1; /* libpcap's end, or the bytes ran out */
            b->dirbits_len = dirbits_len;
            b->d_dirbits = d_dirbits;
            b->ws_bytes = WS_SLOTS(b->n_tiles) + 64 + 8 * TE_WK_SLOT_WORDS * (uint64_t)te_wave_grid();
            if (pipe_grow(t, P, s) < 0)
                goto fail;
            HIPCHK(t, hipMemsetAsync(b->d_ws, 0, WS_STATE, t->stream)); /* err, ticket, both counter sets */
            HIPCHK(t, hipMemsetAsync(b->d_ws + WS_LIST_CNT(b->n_tiles), 0, 8, t->stream));
            HIPCHK(t, hipStreamWaitEvent(t->stream, P->d2h_done[s], 0));
            if (launch(b, -1) != 0) {
                te_seterr(t, "kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
                goto fail;
            }
            if (run_q8(t, b, -1, pkts == 0, NULL, 0, t->stream) < 0)
                goto fail;
            HIPCHK(t, hipMemcpyAsync(b->res_pinned, b->d_ws, WS_STATE, hipMemcpyDeviceToHost, t->stream));
            if (b->last_fgrid)
                HIPCHK(t, hipMemcpyAsync(b->res_pinned + TE_RES_SLOTS, b->d_ws + WS_SLOTS(b->n_tiles),
                                         8 * TE_WK_SLOT_WORDS * (size_t)b->last_fgrid, hipMemcpyDeviceToHost,
                                         t->stream));
            HIPCHK(t, hipEventRecord(P->edit_done[s], t->stream));
            /* a size-preserving config writes each record at its input offset, so the chunk's
               output is its records' bytes: start their D2H behind the edit now, without the
               host's round trip for the results (pipe_finish_chunk checks them and copies
               again only when a replay changed the bytes) */
            if (!b->slot_layout && static_capable(&t->cfg) && !b->has_trim && b->stop_error_pkt < 0 &&
                !getenv("TCPEDIT_HIP_PIPE_NO_EARLY") &&
                pos_early + (b->walk_end - entry_img) <= out_cap) {
                const uint64_t ob_ = b->out_base ? b->out_base : 24, nb_ = b->walk_end - entry_img;
                HIPCHK(t, hipStreamWaitEvent(P->s_d2h, P->edit_done[s], 0));
                HIPCHK(t, hipMemcpyAsync(dst + pos_early, b->d_out + ob_, nb_, hipMemcpyDeviceToHost, P->s_d2h));
                HIPCHK(t, hipEventRecord(P->d2h_done[s], P->s_d2h));
                P->early[s] = pos_early;
                pos_early += nb_;
                P->early_n++;
            } else {
                pos_early = ~0ull >> 1; /* (from here on the results decide every copy) */
            }
            inflight[s] = 1;
            chunk_pkt_base[s] = pkts;
            pkts += b->n_pkts;
            P->first_off[s] = chunk_first;
            P->prev_off[s] = prev_first;
            pipe_anchor(P, chunk_first);
            prev_first = chunk_first;
        }
        if (more && !stopped)
            DIX_INDEX(k + 1);
        /* ---- the previous chunk: results in, D2H to its place ---- */
        const int ps = (k + TE_PIPE_SLOTS - 1) % TE_PIPE_SLOTS;
        if (k > 0 && inflight[ps] == 1) {
            HIPCHK(t, hipEventSynchronize(P->edit_done[ps]));
            inflight[ps] = 2;
            if (pipe_finish_chunk(t, P, ps, chunk_pkt_base[ps], dst, out_cap, &pos, &stopped) < 0)
                goto fail;
        }
        if (stopped || !more)
            break;
    }
    for (int j = 0; j < TE_PIPE_SLOTS; j++) { /* the chunk still in flight */
        const int s = (k + TE_PIPE_SLOTS - j) % TE_PIPE_SLOTS;
        if (inflight[s] == 1) {
            HIPCHK(t, hipEventSynchronize(P->edit_done[s]));
            inflight[s] = 2;
            if (pipe_finish_chunk(t, P, s, chunk_pkt_base[s], dst, out_cap, &pos, &stopped) < 0)
                goto fail;
        }
    }
    HIPCHK(t, hipStreamSynchronize(P->s_d2h));
    if (trace)
        fprintf(stderr, "pipe (device index): %d chunks, %.3f ms, index waits %.3f ms, host-walk fallbacks %d, "
                "early D2H %u (again %u)\n", k + 1, (te_now() - t0) * 1e3, t_wait * 1e3, fallbacks, P->early_n,
                P->early_miss);
    *pos_io = pos;
    free(cst);
#undef DIX_UPLOAD
#undef DIX_INDEX
    return 0;
fail:
    hipStreamSynchronize(P->s_h2d);
    hipStreamSynchronize(t->stream);
    hipStreamSynchronize(P->s_d2h);
    free(cst);
    return -1;
}

static int win_pipe_off(void)
{
    const char *e = getenv("TCPEDIT_HIP_PIPE_NO_WIN");
    return e && *e && *e != '0';
}

/* the window-mode pipeline's chunk starts: C/4 and C/2 (at least 1 MiB) to fill the
   pipeline, C-sized chunks, then halving pieces to drain it -- every chunk but the last a
   multiple of 16 bytes (the head copy moves 16-byte pieces) */
static uint64_t *win_plan(size_t in_len, uint64_t C, uintptr_t addr, int *n_out)
{
    /* (chunk starts 256-byte aligned: 4 KiB and 64 KiB alignment measured the same,
       profiles/r05_e2e_ab.txt) */
    const uint64_t MIN = (uint64_t)1 << 20, A = 256;
    const int cap = (int)((in_len / MIN) + 16);
    uint64_t *st = malloc(sizeof(uint64_t) * (size_t)cap);
    if (!st)
        return NULL;
    int n = 0;
    uint64_t at = 24;
    st[n++] = at;
    while (at < in_len && n < cap - 1) {
        const uint64_t rem = in_len - at;
        uint64_t sz;
        if (n == 1)
            sz = C / 4;
        else if (n == 2)
            sz = C / 2;
        else
            sz = rem > C + C / 2 ? C : rem / 2; /* (the drain halves what is left) */
        if (sz < MIN)
            sz = MIN;
        if (sz > C)
            sz = C;
        /* chunk starts 256-byte aligned in the caller's buffer after the first (the copies
           run slower from and to misaligned addresses) */
        sz = n == 1 ? ((addr + at + sz) & ~(uintptr_t)(A - 1)) - (addr + at) : sz & ~(A - 1);
        if (sz >= rem)
            sz = rem;
        st[n++] = (at += sz);
    }
    st[n - 1] = in_len;
    *n_out = n - 1;
    return st;
}

/* bytes past a window-mode chunk uploaded with it: a record starting in the chunk may end
   there; one that ends further out breaks the chain (the exact pipeline redoes the capture) */
#define TE_PIPE_WIN_MARGIN ((uint64_t)65536)

/* The window-mode pipeline, for the wave lane's size-preserving configs without a tcpprep
 * cache (what tcpedit_batch_run_fused carries): chunk k is the file bytes [cst_k, cst_k+1)
 * uploaded with the next TE_PIPE_WIN_MARGIN bytes and edited in window mode -- the wave lane
 * finds its records itself, the first where the previous chunk's chain ended (read on the
 * device).  Records keep their file offsets, so the chunk's output image, completed with
 * the previous chunk's last record (the check launch copies it), goes down as the same file
 * range.  No host wait per chunk beyond keeping two chunks ahead: the block totals and
 * chain verdicts gather on the device, read once at the end.  Returns 0 (*pos_io: the
 * output's end), 1 (a chunk missed the chain, a chain end or a record the window mode
 * leaves to the exact path: the caller runs the exact pipeline over the whole capture;
 * the same bytes), or -1. */
static int pipe_run_win(tcpedit_t *t, te_pipe_t *P, const uint8_t *img, size_t in_len, uint8_t *dst, size_t out_cap,
                        uint64_t *pos_io, int trace)
{
    const uint64_t C = P->chunk;
    if (in_len > out_cap || in_len < 24 + 16)
        return 1; /* (the copies move whole file ranges) */
    int nch = 0;
    /* a chunk's bytes sit at image offset ORG (the file header is not in the image: the
       window mode starts from the chunk's first record), 256-byte aligned on the device as
       the chunk starts are in the caller's buffers (win_plan) */
    const uint64_t ORG = 256;
    uint64_t *cst = win_plan(in_len, C, (uintptr_t)img, &nch);
    if (!cst) {
        te_seterr(t, "out of memory");
        return -1;
    }
    if (nch > P->nopen && P->nopen < TE_PIPE_SLOTS) { /* (pipe_ready's bound on the chunks) */
        te_seterr(t, "pipeline: %d chunks over %d open slots", nch, P->nopen);
        free(cst);
        return -1;
    }
    const double t0 = te_now();
    if (!P->d_wacc) {
        HIPCHK(t, hipMalloc((void **)&P->d_wacc, 64));
        HIPCHK(t, hipHostMalloc((void **)&P->h_wacc, 64, 0));
    }
    {
        const uint64_t limit_max = ORG + C + 256;
        const uint32_t nwin_max = (uint32_t)((limit_max - ORG + te_win_bytes() - 1) / te_win_bytes());
        for (int s = 0; s < P->nopen; s++) {
            tcpedit_batch_t *b = P->slot[s];
            b->out_cap = C + 256 + TE_PIPE_WIN_MARGIN + ORG;
            if (win_ready(t, b, nwin_max) < 0 || pipe_grow(t, P, s) < 0)
                goto fail;
        }
    }
    HIPCHK(t, hipMemsetAsync(P->d_wacc, 0, 32, t->stream));
    int last = 0;
    /* TCPEDIT_HIP_PIPE_ZC=1 (A/B): the output written by the kernel straight into the
       caller's page-locked buffer over PCIe (its device address) -- no D2H copies, and a
       chunk's last record is written whole by its own launch, so no head copy either.  On
       C2 the kernel's PCIe writes ran at ~34 GB/s and the call took 2.35 ms against 2.18
       with the copies, so the copies stay the default */
    uint8_t *zc = NULL;
    {
        const char *e = getenv("TCPEDIT_HIP_PIPE_ZC");
        void *dp = NULL;
        /* (the stores reach up to 15 bytes past the last record: room for them) */
        if (e && *e == '1' && out_cap >= in_len + 16 && hipHostGetDevicePointer(&dp, dst, 0) == hipSuccess && dp)
            zc = (uint8_t *)dp;
        (void)hipGetLastError();
    }
    /* chunks enqueued ahead of the oldest unfinished edit (TCPEDIT_HIP_PIPE_WIN_AHEAD, A/B):
       the host keeps the streams' cross waits few instead of queueing the whole capture */
    int ahead = 2;
    {
        const char *e = getenv("TCPEDIT_HIP_PIPE_WIN_AHEAD");
        if (e && *e)
            ahead = atoi(e);
    }
    /* TCPEDIT_HIP_PIPE_TIMELINE=1 (diagnostics): timing events per chunk -- upload start and
       end, edit end, download start and end -- printed relative to the first upload */
    enum { TL_H0, TL_H1, TL_E1, TL_D0, TL_D1, TL_N };
    const int tl_on = getenv("TCPEDIT_HIP_PIPE_TIMELINE") != NULL && nch <= 64;
    hipEvent_t tl[64][TL_N];
    double tl_host[64];
    if (tl_on)
        for (int k = 0; k < nch; k++)
            for (int e = 0; e < TL_N; e++)
                HIPCHK(t, hipEventCreate(&tl[k][e]));
    for (int k = 0; k < nch; k++) {
        const int s = k % TE_PIPE_SLOTS, ps = (k + TE_PIPE_SLOTS - 1) % TE_PIPE_SLOTS;
        tcpedit_batch_t *b = P->slot[s], *pb = P->slot[ps];
        if (ahead > 0 && ahead < TE_PIPE_SLOTS && k >= ahead)
            HIPCHK(t, hipEventSynchronize(P->edit_done[(k - ahead) % TE_PIPE_SLOTS]));
        if (tl_on)
            tl_host[k] = te_now() - t0;
        const uint64_t f0 = cst[k], f1 = cst[k + 1];
        const uint64_t fe = f1 + TE_PIPE_WIN_MARGIN < in_len ? f1 + TE_PIPE_WIN_MARGIN : in_len;
        /* upload (the slot's last window kernel has read its input) */
        if (k >= TE_PIPE_SLOTS)
            HIPCHK(t, hipStreamWaitEvent(P->s_h2d, P->edit_done[s], 0));
        if (tl_on)
            HIPCHK(t, hipEventRecord(tl[k][TL_H0], P->s_h2d));
        HIPCHK(t, hipMemcpyAsync(b->d_in + ORG, img + f0, fe - f0, hipMemcpyHostToDevice, P->s_h2d));
        HIPCHK(t, hipEventRecord(P->h2d_done[s], P->s_h2d));
        if (tl_on)
            HIPCHK(t, hipEventRecord(tl[k][TL_H1], P->s_h2d));
        b->in_len = ORG + (fe - f0);
        b->n_tiles = 0;
        b->rec0 = b->out_base = ORG; /* records keep their image offsets */
        b->launches = 0;
        b->gen_hint_ok = 0;
        te_win_req_t q;
        memset(&q, 0, sizeof q);
        q.len = b->in_len;
        q.entry = ORG;
        q.base = ORG;
        q.limit = f1 >= in_len ? b->in_len : ORG + (f1 - f0);
        q.nwin = (uint32_t)((q.limit - q.base + te_win_bytes() - 1) / te_win_bytes());
        q.entry_ptr = k ? (const uint64_t *)(pb->d_win + WIN_TOT_OFF(pb->win_cap)) : NULL;
        q.entry_sub = k ? f0 - cst[k - 1] : 0; /* the previous chunk's image is that much earlier */
        q.acc = P->d_wacc;
        q.prev_out = k && !zc ? pb->d_out : NULL;
        q.head_max = ORG + TE_PIPE_WIN_MARGIN;
        q.org = ORG;
        q.out = zc ? zc + f0 - ORG : NULL; /* (image offset x is file offset f0 + x - ORG) */
        /* the window kernel: after the upload, and after the slot's last output copy */
        HIPCHK(t, hipStreamWaitEvent(t->stream, P->h2d_done[s], 0));
        if (!zc)
            HIPCHK(t, hipStreamWaitEvent(t->stream, P->d2h_done[s], 0));
        b->win_req = &q;
        const int lr = launch(b, -1);
        b->win_req = NULL;
        if (lr != 0) {
            te_seterr(t, "window-mode launch failed: %s", hipGetErrorString(hipGetLastError()));
            goto fail;
        }
        HIPCHK(t, hipEventRecord(P->edit_done[s], t->stream));
        if (tl_on)
            HIPCHK(t, hipEventRecord(tl[k][TL_E1], t->stream));
        if (!zc) { /* the chunk's file range down, behind its edit */
            HIPCHK(t, hipStreamWaitEvent(P->s_d2h, P->edit_done[s], 0));
            if (tl_on)
                HIPCHK(t, hipEventRecord(tl[k][TL_D0], P->s_d2h));
            HIPCHK(t, hipMemcpyAsync(dst + f0, b->d_out + ORG, f1 - f0, hipMemcpyDeviceToHost, P->s_d2h));
            HIPCHK(t, hipEventRecord(P->d2h_done[s], P->s_d2h));
            if (tl_on)
                HIPCHK(t, hipEventRecord(tl[k][TL_D1], P->s_d2h));
        }
        last = s;
    }
    {
        tcpedit_batch_t *b = P->slot[last];
        HIPCHK(t, hipMemcpyAsync(P->h_wacc, P->d_wacc, 32, hipMemcpyDeviceToHost, t->stream));
        HIPCHK(t, hipMemcpyAsync(P->h_wacc + 4, b->d_win + WIN_TOT_OFF(b->win_cap), 8,
                                 hipMemcpyDeviceToHost, t->stream));
        HIPCHK(t, hipStreamSynchronize(t->stream));
        HIPCHK(t, hipStreamSynchronize(P->s_d2h));
    }
    if (trace)
        fprintf(stderr, "pipe (window mode%s): %d chunks, %.3f ms, verdict %llu\n", zc ? ", output over PCIe" : "",
                nch, (te_now() - t0) * 1e3, (unsigned long long)P->h_wacc[3]);
    if (tl_on) {
        for (int k = 0; k < nch; k++) {
            float v[TL_N] = {0};
            for (int e = 0; e < TL_N; e++)
                if (!zc || e < TL_D0)
                    (void)hipEventElapsedTime(&v[e], tl[0][TL_H0], tl[k][e]);
            fprintf(stderr, "tl chunk %2d %6.2f MiB: host %.3f | up %.3f-%.3f | edit end %.3f | down %.3f-%.3f ms\n",
                    k, (cst[k + 1] - cst[k]) / 1048576.0, tl_host[k] * 1e3, v[TL_H0], v[TL_H1], v[TL_E1], v[TL_D0],
                    v[TL_D1]);
        }
        for (int k = 0; k < nch; k++)
            for (int e = 0; e < TL_N; e++)
                hipEventDestroy(tl[k][e]);
    }
    {
        const uint64_t *acc = P->h_wacc;
        const uint64_t f0 = cst[nch - 1];
        const uint64_t end = f0 + acc[4] - ORG; /* the last chunk's chain end, as a file offset */
        free(cst);
        if (acc[3] || acc[1] != end - 24 || end > in_len) { /* (the records and the chain must agree) */
            if (trace)
                fprintf(stderr, "pipe (window mode): missed -- verdict %llu, chain end %llu, records end %llu of %zu;"
                                " the exact pipeline redoes the capture\n",
                        (unsigned long long)acc[3], (unsigned long long)end, (unsigned long long)(acc[1] + 24),
                        in_len);
            return 1;
        }
        *pos_io = end;
        t->pub.runtime.packetnum += acc[0];
        t->pub.runtime.total_bytes += acc[1];
        t->pub.runtime.pkts_edited += acc[2];
    }
    return 0;
fail:
    hipStreamSynchronize(P->s_h2d);
    hipStreamSynchronize(t->stream);
    hipStreamSynchronize(P->s_d2h);
    free(cst);
    return -1;
}

int tcpedit_rewrite_pcap_pipelined(tcpedit_t *t, const void *in, size_t in_len, const void *cache, size_t cache_len,
                                   void *out, size_t out_cap, size_t *out_len, size_t chunk_bytes)
{
    if (t && in && te_is_pcapng((const uint8_t *)in, in_len)) { /* as libpcap's reader delivers it */
        uint8_t *ng = NULL;
        size_t ng_len = 0;
        char e[256];
        if (te_pcapng_to_pcap((const uint8_t *)in, in_len, &ng, &ng_len, e, sizeof e) < 0) {
            te_seterr(t, "%s", e);
            return TCPEDIT_ERROR;
        }
        const int rc = tcpedit_rewrite_pcap_pipelined(t, ng, ng_len, cache, cache_len, out, out_cap, out_len,
                                                      chunk_bytes);
        free(ng);
        return rc;
    }
    const uint8_t *img = in;
    uint8_t *dst = out;
    uint8_t *d_dirbits = NULL;
    uint64_t dirbits_len = 0;
    int reg_in = 0, reg_out = 0, rc = TCPEDIT_ERROR, inflight[TE_PIPE_SLOTS] = {0};
    uint64_t pos = 24, pkts = 0, chunk_pkt_base[TE_PIPE_SLOTS] = {0};
    int stopped = 0; /* a hard error or libpcap's stop ended the walk */
    if (out_len)
        *out_len = 0;
    if (!t || !img || !dst || !out_len || out_cap < 24)
        return TCPEDIT_ERROR;
    if (te_ensure_cfg(t) < 0)
        return TCPEDIT_ERROR;
    if (in_len < 24) {
        te_seterr(t, "pcap image too short");
        return TCPEDIT_ERROR;
    }
    if (chunk_bytes == 0) {
        const size_t tenth = (in_len / 10 + ((size_t)1 << 20) - 1) & ~(((size_t)1 << 20) - 1);
        chunk_bytes = tenth < TE_PIPE_CHUNK_MIN ? TE_PIPE_CHUNK_MIN : tenth > TE_PIPE_CHUNK_MAX ? TE_PIPE_CHUNK_MAX : tenth;
    }
    if (chunk_bytes < ((size_t)1 << 20))
        chunk_bytes = (size_t)1 << 20; /* >= any record (16 + 262144 B) */
    chunk_bytes = (chunk_bytes + 15) & ~(size_t)15;
    /* the chunks the capture can be cut into: every chunk but the last holds >= 1 MiB of the
       window plan or >= chunk - one largest record of a record-cut plan (>= 1 MiB - 262,160) */
    const int want = (int)((in_len > 24 ? in_len - 24 : 0) / (((size_t)1 << 20) - 262160u) + 2);
    if (te_upload_cfg(t) < 0 || pipe_ready(t, chunk_bytes, want) < 0)
        return TCPEDIT_ERROR;
    te_pipe_t *P = t->pipe;
    {
        uint32_t magic, lt;
        memcpy(&magic, img, 4);
        const int sw = magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u;
        if (magic != 0xa1b2c3d4u && magic != 0xa1b23c4du && !sw) {
            te_seterr(t, "not a pcap file (magic 0x%08x)", magic);
            return TCPEDIT_ERROR;
        }
        lt = te_linktype_dlt(rd32(img + 20, sw) & 0x03ffffffu);
        if (lt != (uint32_t)t->dlt) {
            te_seterr(t, "pcap linktype %u does not match the context DLT %d", lt, t->dlt);
            return TCPEDIT_ERROR;
        }
    }
    memcpy(P->hdr, img, 24);
    {
        /* pcap_open_dead(out_dlt, 65535) + pcap_dump_open (tcprewrite.c:124,147) */
        out_header(t, dst);
    }
    if (cache) {
        const uint8_t *cd;
        if (te_check_decoder_cfg(t, 1) < 0)
            return TCPEDIT_ERROR;
        if (cache_data(t, (const uint8_t *)cache, cache_len, &cd, &dirbits_len) < 0)
            return TCPEDIT_ERROR;
        HIPCHK(t, hipMalloc((void **)&d_dirbits, dirbits_len + 16));
        HIPCHK(t, hipMemcpy(d_dirbits, cd, dirbits_len, hipMemcpyHostToDevice));
    } else if (t->cfg.n_cidrmap1 && t->have[OPT_ENDPOINTS]) {
        te_seterr(t, "--endpoints requires a tcpprep cache file");
        return TCPEDIT_ERROR;
    }
    /* page-lock the caller's buffers for the call: the copies then DMA straight from / to
       them (an already locked buffer is used as is; an unlockable one is copied through
       the driver's staging, which is slower but the same bytes) */
    const int trace = getenv("TCPEDIT_HIP_PIPE_TRACE") != NULL;
    double t_start = te_now(), t_reg = 0, t_index = 0, t_wait = 0;
    if (!host_locked(img)) {
        reg_in = hipHostRegister((void *)img, in_len, hipHostRegisterDefault) == hipSuccess;
        (void)hipGetLastError();
    }
    if (!host_locked(dst)) {
        reg_out = hipHostRegister(dst, out_cap, hipHostRegisterDefault) == hipSuccess;
        (void)hipGetLastError();
    }
    t_reg = te_now() - t_start;

    {   /* the wave lane's configs: the record index on the device */
        tcpedit_batch_t *b0 = P->slot[0];
        uint32_t magic;
        memcpy(&magic, img, 4);
        int dix = !pipe_index_host_env();
        for (int s = 0; s < P->nopen; s++) {
            tcpedit_batch_t *bs = P->slot[s];
            bs->swapped = magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u;
            bs->nsec = magic == 0xa1b23c4du || magic == 0x4d3cb2a1u;
            te_walk_t proto;
            cut_setup(t, bs, &proto, img + 24, in_len - 24, P->chunk);
            dix &= bs->cut_device_ok;
        }
        if (dix && b0->fast_kind == TE_FAST_WAVE && !b0->slot_layout && !d_dirbits && !b0->swapped && !b0->nsec &&
            static_capable(&t->cfg) && fast_capable(&t->cfg) && !fast_lane_off() && !win_pipe_off()) {
            /* the window mode: no index passes and no host wait per chunk */
            const int r = pipe_run_win(t, P, img, in_len, dst, out_cap, &pos, trace);
            if (r < 0)
                goto fail;
            if (r == 0) {
                *out_len = pos;
                rc = TCPEDIT_OK;
                goto out;
            }
            t->pipe_fallbacks++;
            pos = 24; /* (the exact pipeline below redoes the capture) */
        }
        if (dix && b0->fast_kind == TE_FAST_WAVE) {
            /* scratch for huge records, sized for the worst chunk (the index places them) */
            for (int s = 0; s < P->nopen; s++) {
                const uint64_t need = (uint64_t)chunk_bytes + TE_PIPE_MARGIN + (chunk_bytes + TE_PIPE_MARGIN) / 8 + 65536;
                if (P->d_scratch_alloc[s] < need) {
                    hipFree(P->slot[s]->d_scratch);
                    P->slot[s]->d_scratch = NULL;
                    HIPCHK(t, hipMalloc((void **)&P->slot[s]->d_scratch, need));
                    P->d_scratch_alloc[s] = need;
                }
            }
            if (pipe_run_dix(t, P, img, in_len, dst, out_cap, d_dirbits, dirbits_len, &pos, trace) < 0)
                goto fail;
            *out_len = pos;
            rc = t->pipe_err ? TCPEDIT_ERROR : TCPEDIT_OK;
            goto out;
        }
    }

    uint64_t off = 24; /* file offset of the next chunk's first record */
    uint64_t prev_first = ~0ull;
    P->img = img;
    P->nanchor = 0; /* (this call's capture) */
    int k = 0;
    for (;; k++) {
        const int s = k % TE_PIPE_SLOTS;
        tcpedit_batch_t *b = P->slot[s];
        /* ---- finish the chunk that held this slot: its results, then its D2H ---- */
        double tw = te_now();
        if (inflight[s]) {
            HIPCHK(t, hipEventSynchronize(P->edit_done[s]));
            inflight[s] = 0;
        }
        if (stopped || off + 16 > in_len)
            break;
        if (!b) { /* (pipe_ready's bound on the chunks) */
            te_seterr(t, "pipeline: chunk %d over %d open slots", k, P->nopen);
            goto fail_drain;
        }
        /* ---- index the next chunk into the slot (its pinned arrays are free once the
               H2D that read them is done) ---- */
        HIPCHK(t, hipEventSynchronize(P->h2d_done[s]));
        double ti = te_now();
        t_wait += ti - tw;
        const size_t avail = in_len - off, take = avail < chunk_bytes ? avail : chunk_bytes;
        /* the chunk's bytes go up while the host walks them (the slot's input is free: its
           last edit is done); the walk decides how many of them are whole records */
        HIPCHK(t, hipMemcpyAsync(b->d_in, P->hdr, 24, hipMemcpyHostToDevice, P->s_h2d));
        HIPCHK(t, hipMemcpyAsync(b->d_in + 24, img + off, take, hipMemcpyHostToDevice, P->s_h2d));
        b->pkt_base = pkts;
        b->launches = 0;
        b->gen_hint_ok = 0;
        b->rec0 = b->out_base = 0;
        free(b->slots_host);
        b->slots_host = NULL;
        if (index_image(t, b, img, img + off, take + 24) < 0)
            goto fail;
        t_index += te_now() - ti;
        if (b->n_pkts == 0) { /* the walk stopped at the chunk's first record */
            stopped = 1;
            if (b->stop_error_pkt >= 0) {
                te_seterr(t, TE_READER_ERR, (long long)(pkts + 1));
                goto fail_drain;
            }
            break;
        }
        if (b->walk_stop || (b->walk_end - 24 < take && take == avail)) /* libpcap's end or an error */
            stopped = 1;
        b->dirbits_len = dirbits_len;
        b->d_dirbits = d_dirbits;
        b->ws_bytes = WS_SLOTS(b->n_tiles) + 64 + 8 * TE_WK_SLOT_WORDS * (uint64_t)te_wave_grid();
        if (pipe_grow(t, P, s) < 0)
            goto fail_drain;
        const size_t rec_bytes = (size_t)(b->walk_end - 24);
        /* ---- H2D: header, records, index; the kernel stream waits for it and for the
               D2H of the chunk this slot held before ---- */
        HIPCHK(t, hipMemcpyAsync(b->d_tiles, b->tiles, sizeof(te_tile_t) * b->n_tiles, hipMemcpyHostToDevice,
                                 P->s_h2d));
        b->tcut_ok = 0;
        HIPCHK(t, hipMemcpyAsync(b->d_pkt_rel, b->pkt_rel, sizeof(uint16_t) * b->n_pkts, hipMemcpyHostToDevice,
                                 P->s_h2d));
        HIPCHK(t, hipMemsetAsync(b->d_ws, 0, WS_STATE, P->s_h2d)); /* err, ticket, both counter sets */
        HIPCHK(t, hipMemsetAsync(b->d_ws + WS_LIST_CNT(b->n_tiles), 0, 8, P->s_h2d));
        HIPCHK(t, hipEventRecord(P->h2d_done[s], P->s_h2d));
        HIPCHK(t, hipStreamWaitEvent(t->stream, P->h2d_done[s], 0));
        HIPCHK(t, hipStreamWaitEvent(t->stream, P->d2h_done[s], 0));
        /* ---- edit ---- */
        if (launch(b, -1) != 0) {
            te_seterr(t, "kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
            goto fail_drain;
        }
        /* stale static-buffer reads (Q8): the replay kernel reads the listed count on the
           device and returns at once when it is 0; chunk 0 starts at the capture's start */
        if (run_q8(t, b, -1, pkts == 0, NULL, 0, t->stream) < 0)
            goto fail_drain;
        HIPCHK(t, hipMemcpyAsync(b->res_pinned, b->d_ws, WS_STATE, hipMemcpyDeviceToHost, t->stream));
        if (b->last_fgrid)
            HIPCHK(t, hipMemcpyAsync(b->res_pinned + TE_RES_SLOTS, b->d_ws + WS_SLOTS(b->n_tiles),
                                     8 * TE_WK_SLOT_WORDS * (size_t)b->last_fgrid, hipMemcpyDeviceToHost, t->stream));
        HIPCHK(t, hipEventRecord(P->edit_done[s], t->stream));
        inflight[s] = 1;
        chunk_pkt_base[s] = pkts;
        pkts += b->n_pkts;
        P->first_off[s] = off;
        P->prev_off[s] = prev_first;
        pipe_anchor(P, off);
        prev_first = off;
        off += rec_bytes;

        /* ---- the previous chunk: results in, D2H to its place ---- */
        const int ps = (k + TE_PIPE_SLOTS - 1) % TE_PIPE_SLOTS;
        if (k > 0 && inflight[ps] == 1) {
            HIPCHK(t, hipEventSynchronize(P->edit_done[ps]));
            inflight[ps] = 2; /* results read, D2H issued */
            if (pipe_finish_chunk(t, P, ps, chunk_pkt_base[ps], dst, out_cap, &pos, &stopped) < 0)
                goto fail_drain;
        }
    }
    /* the chunks still in flight, in order */
    for (int j = 1; j <= TE_PIPE_SLOTS; j++) {
        const int s = (k + j) % TE_PIPE_SLOTS;
        if (inflight[s] == 1) {
            HIPCHK(t, hipEventSynchronize(P->edit_done[s]));
            inflight[s] = 2;
            if (pipe_finish_chunk(t, P, s, chunk_pkt_base[s], dst, out_cap, &pos, &stopped) < 0)
                goto fail_drain;
        }
    }
    HIPCHK(t, hipStreamSynchronize(P->s_d2h));
    *out_len = pos;
    rc = t->pipe_err ? TCPEDIT_ERROR : TCPEDIT_OK;
    if (trace)
        fprintf(stderr, "pipe: %d chunks, %.3f ms total: register %.3f, index %.3f, waits %.3f (reg in %d out %d)\n",
                k, (te_now() - t_start) * 1e3, t_reg * 1e3, t_index * 1e3, t_wait * 1e3, reg_in, reg_out);
    goto out;
fail_drain:
    hipStreamSynchronize(P->s_h2d);
    hipStreamSynchronize(t->stream);
    hipStreamSynchronize(P->s_d2h);
fail:
    rc = TCPEDIT_ERROR;
out:
    if (reg_in)
        hipHostUnregister((void *)img);
    if (reg_out)
        hipHostUnregister(dst);
    if (d_dirbits) {
        hipStreamSynchronize(t->stream);
        hipFree(d_dirbits);
    }
    for (int s = 0; P && s < TE_PIPE_SLOTS; s++)
        if (P->slot[s])
            P->slot[s]->d_dirbits = NULL;
    t->pipe_err = 0;
    return rc;
}

/* ------------------------------------------------------------------------- */
/* reference interface                                                       */
/* ------------------------------------------------------------------------- */
int tcpedit_init(tcpedit_t **out, int dlt)
{
    tcpedit_t *t = calloc(1, sizeof(*t));
    *out = t;
    if (!t)
        return TCPEDIT_ERROR;
    t->dlt = dlt;
    t->device = g_device;
    /* defaults until post_args (tcpedit.c:382-394) */
    te_cfg_defaults(&t->cfg, dlt);
    t->fuzz_factor = 8; /* DEFAULT_FUZZ_FACTOR */
    t->pub.runtime.dlt1 = t->pub.runtime.dlt2 = dlt;
    t->dev_dirty = 1;
    te_sync_pub(t);
    if (te_decoder_of(dlt) < 0) {
        te_seterr(t, "No DLT plugin available for source DLT: 0x%x (this build: EN10MB, LINUX_SLL, LINUX_SLL2, "
                     "RAW, NULL, LOOP, PPP_SERIAL, C_HDLC, JUNIPER_ETHER, IEEE802_11, IEEE802_11_RADIO)", dlt);
        return TCPEDIT_ERROR;
    }
    return TCPEDIT_OK;
}

/* parse_args.c:34-254.  The option source: the store (tcpedit_parse_args /
 * tcpedit_set_option), else the calling tool's AutoOpts option set (te_autoopts.c),
 * else the setters' values; with none of them there is nothing to derive from, and a
 * run would silently apply no edits, so it is an error. */
int tcpedit_post_args(tcpedit_t *t)
{
    if (!t)
        return TCPEDIT_ERROR;
    t->pub.runtime.errstr[0] = 0;
    if (!(t->opt_src & TE_SRC_STORE)) {
        const int r = te_autoopts_import(t);
        if (r < 0)
            return TCPEDIT_ERROR;
        if (r == 0) {
            if (t->opt_src & TE_SRC_SETTERS) { /* the setter API (tcpedit_api.h) stands alone */
                t->post_args_done = 1;
                te_sync_pub(t);
                return TCPEDIT_OK;
            }
            te_seterr(t, "tcpedit_post_args: no option source -- no AutoOpts option set "
                         "(tcprewriteOptions/tcpreplayOptions/tcpbridgeOptions) in this process, and "
                         "neither tcpedit_parse_args/tcpedit_set_option nor a tcpedit_set_* setter was called");
            return TCPEDIT_ERROR;
        }
    }
    return te_derive_cfg(t) < 0 ? TCPEDIT_ERROR : TCPEDIT_OK;
}

/* the derivation a run needs, once: post_args, or (setter API) the setters' values as
   they stand */
int te_ensure_cfg(tcpedit_t *t)
{
    if (t->post_args_done)
        return 0;
    if ((t->opt_src & TE_SRC_SETTERS) && !(t->opt_src & TE_SRC_STORE)) {
        t->post_args_done = 1;
        te_sync_pub(t);
        return 0;
    }
    return tcpedit_post_args(t) < 0 ? -1 : 0;
}

int tcpedit_validate(tcpedit_t *t)
{
    if (!t)
        return TCPEDIT_ERROR;
    t->pub.validated = 1;
    return TCPEDIT_OK;
}

char *tcpedit_geterr(tcpedit_t *t) { return t ? t->pub.runtime.errstr : NULL; }
char *tcpedit_getwarn(tcpedit_t *t) { return t ? t->pub.runtime.warnstr : NULL; }

int tcpedit_checkerror(tcpedit_t *t, int rcode, const char *prefix)
{
    switch (rcode) {
    case TCPEDIT_OK:
    case TCPEDIT_ERROR:
        return rcode;
    case TCPEDIT_SOFT_ERROR:
        fprintf(stderr, prefix ? "Error %s: %s\n" : "Error%s: %s\n", prefix ? prefix : "", tcpedit_geterr(t));
        break;
    case TCPEDIT_WARN:
        fprintf(stderr, prefix ? "Warning %s: %s\n" : "Warning%s: %s\n", prefix ? prefix : "", tcpedit_getwarn(t));
        return TCPEDIT_OK;
    default:
        break;
    }
    return TCPEDIT_ERROR;
}

int tcpedit_get_output_dlt(tcpedit_t *t)
{
    if (!t)
        return -1;
    if (te_ensure_cfg(t) < 0)
        return -1;
    return t->cfg.out_linktype; /* tcpedit_dlt_output_dlt (dlt_plugins.c:268-283) */
}

int tcpedit_get_dev_cfg(tcpedit_t *t, void *out, size_t len, uint16_t *portlut)
{
    if (!t || !out || len < sizeof(te_dev_cfg_t))
        return -1;
    memcpy(out, &t->cfg, sizeof(te_dev_cfg_t));
    ((te_dev_cfg_t *)out)->slot_head = te_slot_head(&t->cfg);
    if (portlut) {
        for (int p = 0; p < 65536; p++)
            portlut[p] = t->portlut ? t->portlut[p] : (uint16_t)p;
    }
    return (int)sizeof(te_dev_cfg_t);
}
uint64_t tcpedit_get_total_bytes(tcpedit_t *t) { return t ? t->pub.runtime.total_bytes : 0; }
uint64_t tcpedit_get_pkts_edited(tcpedit_t *t) { return t ? t->pub.runtime.pkts_edited : 0; }

/* tcpedit_l3data / tcpedit_l3proto: L2 walk of an (un)edited frame; these are
 * the DLT plugins' l3 accessors (dlt_en10mb_get_layer3 / _proto), pure header
 * inspection used by callers such as fragroute (tcprewrite.c:338) */
static int host_l2(const unsigned char *p, int n, uint16_t *proto)
{
    if (n <= 18)
        return -1;
    uint32_t off = 14;
    uint16_t et = (uint16_t)((p[12] << 8) | p[13]);
    for (int guard = 0; guard < 4096; guard++) {
        if (et == 0x8100 || et == 0x88A8 || et == 0x9100) {
            if ((uint32_t)n < off + 4)
                return -1;
            et = (uint16_t)((p[off + 2] << 8) | p[off + 3]);
            off += 4;
        } else if (et == 0x8847 || et == 0x8848) {
            int bos = 0;
            uint32_t lab = off;
            while (!bos) {
                if (off + 4 > (uint32_t)n)
                    return -1;
                lab = off;
                bos = (p[off + 2] & 1) != 0;
                if ((((uint32_t)p[off] << 12) | ((uint32_t)p[off + 1] << 4) | (p[off + 2] >> 4)) == 13)
                    return -1;
                off += 4;
            }
            if (lab + 5 > (uint32_t)n)
                return -1;
            uint8_t nib = p[lab + 4] >> 4;
            if (nib == 4)
                et = 0x0800;
            else if (nib == 6)
                et = 0x86DD;
            else if (nib == 0) {
                if (off + 18 > (uint32_t)n)
                    return -1;
                off += 4;
                et = (uint16_t)((p[off + 12] << 8) | p[off + 13]);
                off += 14;
            } else
                return -1;
        } else
            break;
    }
    if (et < 1536)
        return -1;
    *proto = et;
    return (int)off;
}

const unsigned char *tcpedit_l3data(tcpedit_t *t, tcpedit_coder code, unsigned char *packet, int pktlen)
{
    (void)t;
    (void)code;
    uint16_t pr;
    int l2 = host_l2(packet, pktlen, &pr);
    if (l2 < 0 || pktlen <= l2)
        return NULL;
    return packet + l2;
}

int tcpedit_l3proto(tcpedit_t *t, tcpedit_coder code, const unsigned char *packet, int pktlen)
{
    (void)t;
    (void)code;
    uint16_t pr;
    if (pktlen < 14 || host_l2(packet, pktlen, &pr) < 0)
        return 0xffff; /* ntohs(TCPEDIT_ERROR) (tcpedit.c:651) */
    return pr;
}

/* ---- DLT plugin API (plugins_api.h:29-78) ---------------------------------- */
int tcpedit_dlt_post_args(tcpedit_t *t) { return tcpedit_post_args(t); }

tcpeditdlt_t *tcpedit_dlt_init(tcpedit_t *t, int srcdlt)
{
    if (!t)
        return NULL;
    if (srcdlt != 1) {
        te_seterr(t, "No DLT plugin available for source DLT: 0x%x", srcdlt);
        return NULL;
    }
    te_sync_pub(t);
    return &t->dltc;
}

int tcpedit_dlt_post_init(tcpeditdlt_t *ctx) { return ctx ? TCPEDIT_OK : TCPEDIT_ERROR; }
void tcpedit_dlt_cleanup(tcpeditdlt_t *ctx) { (void)ctx; /* owned by the tcpedit context */ }

int tcpedit_dlt_output_dlt(tcpeditdlt_t *ctx)
{
    return ctx ? tcpedit_get_output_dlt(ctx->tcpedit) : -1;
}

int tcpedit_dlt_src(tcpeditdlt_t *ctx) { return ctx ? ctx->decoder_dlt : -1; }
int tcpedit_dlt_dst(tcpeditdlt_t *ctx) { return ctx ? ctx->encoder_dlt : -1; }

/* the L2 walks of the plugins this build decodes with (en10mb: get_l2len_protocol) */
int tcpedit_dlt_l2len(tcpeditdlt_t *ctx, int dlt, const unsigned char *packet, const int pktlen)
{
    uint16_t pr;
    if (!ctx || !packet)
        return -1;
    if (dlt != 1) {
        te_seterr(ctx->tcpedit, "Unable to find plugin for DLT 0x%04x", dlt);
        return -1;
    }
    const int l2 = pktlen < 14 ? -1 : host_l2(packet, pktlen, &pr);
    if (l2 < 0 || pktlen < l2) {
        te_seterr(ctx->tcpedit, "Packet length %d is to short to contain a layer 2 header for DLT 0x%04x", pktlen,
                  dlt);
        return -1;
    }
    return l2;
}

int tcpedit_dlt_proto(tcpeditdlt_t *ctx, int dlt, const unsigned char *packet, const int pktlen)
{
    uint16_t pr;
    if (!ctx || !packet)
        return -1;
    if (dlt != 1) {
        te_seterr(ctx->tcpedit, "Unable to find plugin for DLT 0x%04x", dlt);
        return -1;
    }
    if (pktlen < 14 || host_l2(packet, pktlen, &pr) < 0)
        return TCPEDIT_ERROR;
    return (int)(uint16_t)((pr >> 8) | (pr << 8)); /* htons(ether_type) (en10mb.c:762) */
}

unsigned char *tcpedit_dlt_l3data(tcpeditdlt_t *ctx, int dlt, unsigned char *packet, const int pktlen)
{
    if (!ctx || dlt != 1)
        return NULL;
    return (unsigned char *)tcpedit_l3data(ctx->tcpedit, BEFORE_PROCESS, packet, pktlen);
}

/* tcpedit_packet's one-record batch, allocated once per context at the largest record
 * (MAXPACKET, defines.h.in:177-182): no device allocation or free per call */
#define TE_ONE_IN (24 + 16 + 262166 + 64)
#define TE_ONE_OUT (24 + 16 + 262166 + 1024 + 64)
static tcpedit_batch_t *one_ready(tcpedit_t *t)
{
    if (t->one)
        return t->one;
    if (te_dev_ready(t) < 0)
        return NULL;
    tcpedit_batch_t *b = calloc(1, sizeof(*b));
    if (!b)
        return NULL;
    b->ctx = t;
    b->idx_pinned = 1;
    b->idx_cap_pkts = b->idx_cap_tiles = 2;
    HIPCHK(t, hipHostMalloc((void **)&b->tiles, sizeof(te_tile_t) * 2, 0));
    HIPCHK(t, hipHostMalloc((void **)&b->pkt_rel, sizeof(uint16_t) * 2, 0));
    HIPCHK(t, hipHostMalloc((void **)&b->one_img, TE_ONE_IN + TE_ONE_OUT, 0));
    HIPCHK(t, hipMalloc((void **)&b->d_in, TE_ONE_IN));
    HIPCHK(t, hipMalloc((void **)&b->d_out, TE_ONE_OUT));
    HIPCHK(t, hipMalloc((void **)&b->d_status, 16));
    HIPCHK(t, hipMalloc((void **)&b->d_scratch, 262144 + 2048));
    HIPCHK(t, hipMalloc((void **)&b->d_tiles, sizeof(te_tile_t) * 2));
    HIPCHK(t, hipMalloc((void **)&b->d_pkt_rel, sizeof(uint16_t) * 2));
    HIPCHK(t, hipMalloc((void **)&b->d_tile_list, sizeof(uint32_t) * 2));
    b->q8_cap = 2;
    b->q8_defer = 1;
    HIPCHK(t, hipMalloc((void **)&b->d_q8, 16 * 2));
    HIPCHK(t, hipMalloc((void **)&b->d_q8_init, 262144 + 64));
    b->ws_bytes = WS_SLOTS(1) + 64 + 8 * TE_WK_SLOT_WORDS * (uint64_t)te_wave_grid();
    HIPCHK(t, hipMalloc((void **)&b->d_ws, b->ws_bytes));
    HIPCHK(t, hipEventCreate(&b->ev0));
    HIPCHK(t, hipEventCreate(&b->ev1));
    t->one = b;
    return b;
fail:
    tcpedit_batch_close(b);
    return NULL;
}

/* ---- tcpedit_packet's resident server (te_packet_server) ----
 * One block stays on the device and serves tcpedit_packet calls through host-mapped
 * fine-grained memory: the record goes into the mapped input image, the request words
 * and seq are stored (release), the host spins on done.  No launch, copy or stream sync
 * per call.  The kernel leaves after TE_SRV_IDLE_TICKS without a request (and is launched
 * again by the next call), when the context's config changes, and at tcpedit_close / exit.
 * TCPEDIT_HIP_PACKET_SERVER=0 keeps the launch-per-call path (A/B). */
#define TE_SRV_IN (24 + 16 + TE_SLOT_BYTES + 64)
#define TE_SRV_OUT (24 + 16 + TE_SLOT_BYTES + 1024)
#define TE_SRV_IDLE_TICKS 5000000ull /* 50 ms of the 100 MHz real-time clock */
#define TE_SRV_DECLINED (-100)       /* the record goes the launch-per-call way */
struct te_srv_s {
    hipStream_t stream;
    te_srv_ctl_t *ctl, *d_ctl;
    uint8_t *in, *d_in, *out, *d_out;
    uint8_t *d_scratch;
    te_dev_cfg_t *d_cfg;
    te_dev_cfg_t cfg;        /* the config the running kernel holds (skip_soft_errors 0) */
    const uint16_t *portlut; /* ... its device port table ... */
    const uint16_t *hportlut; /* ... built from this host table */
    int running;             /* launched and not yet seen leaving */
    int broken;              /* it stopped answering: the launch-per-call path from now on */
    int stuck;               /* it did not leave when stopped: never synced, its buffers never freed */
    uint32_t seq;
};

/* live servers, stopped at exit (a resident kernel must not outlive the mappings it polls) */
#define TE_SRV_MAX 256
static te_srv_t *te_srv_live[TE_SRV_MAX];
static pthread_mutex_t te_srv_mu = PTHREAD_MUTEX_INITIALIZER;
static int te_srv_atexit_done;

/* stop the resident kernel: raise stop, wait (bounded) for it to store alive = 0, then
   sync its stream.  A kernel that never leaves (a broken server, stuck in its tile body)
   is reported and its stream is not synced -- tcpedit_close and exit must not hang on it;
   its mappings are then leaked, not freed under it (srv_free) */
/* (tests: the path of a kernel that never leaves; read once) */
static int srv_test_stuck(void)
{
    static int v = -1;
    if (v < 0)
        v = getenv("TCPEDIT_HIP_SRV_TEST_STUCK") != NULL;
    return v;
}

static int srv_stop(te_srv_t *S)
{
    if (!S->running)
        return 0;
    if (S->stuck) /* it did not leave the last time: do not wait for it again */
        return -1;
    __atomic_store_n(&S->ctl->stop, 1u, __ATOMIC_RELEASE);
    const double t0 = te_now();
    const int test_stuck = srv_test_stuck();
    while (!test_stuck && __atomic_load_n(&S->ctl->alive, __ATOMIC_ACQUIRE)) {
        if (te_now() - t0 > 2.0) {
            fprintf(stderr, "tcpedit: the packet server kernel did not leave in 2 s; its buffers are leaked\n");
            S->stuck = 1;
            return -1;
        }
        __builtin_ia32_pause();
    }
    if (test_stuck) {
        fprintf(stderr, "tcpedit: the packet server kernel did not leave in 2 s; its buffers are leaked\n");
        S->stuck = 1;
        return -1;
    }
    hipStreamSynchronize(S->stream);
    S->running = 0;
    S->ctl->stop = 0;
    return 0;
}

static void srv_stop_all(void)
{
    pthread_mutex_lock(&te_srv_mu);
    for (int i = 0; i < TE_SRV_MAX; i++)
        if (te_srv_live[i])
            srv_stop(te_srv_live[i]);
    pthread_mutex_unlock(&te_srv_mu);
}

static void srv_free(tcpedit_t *t)
{
    te_srv_t *S = t->srv;
    if (!S)
        return;
    pthread_mutex_lock(&te_srv_mu);
    for (int i = 0; i < TE_SRV_MAX; i++)
        if (te_srv_live[i] == S)
            te_srv_live[i] = NULL;
    pthread_mutex_unlock(&te_srv_mu);
    if (S->stream && srv_stop(S) < 0) { /* still running: leave it its mappings */
        t->srv = NULL;
        return;
    }
    if (S->ctl)
        hipHostFree(S->ctl);
    if (S->in)
        hipHostFree(S->in);
    if (S->out)
        hipHostFree(S->out);
    hipFree(S->d_scratch);
    hipFree(S->d_cfg);
    if (S->stream)
        hipStreamDestroy(S->stream);
    free(S);
    t->srv = NULL;
}

static int srv_enabled(void)
{
    const char *e = getenv("TCPEDIT_HIP_PACKET_SERVER");
    return !(e && e[0] == '0');
}

static int srv_launch(tcpedit_t *t, te_srv_t *S, uint32_t start_seq)
{
    te_srv_launch_t L;
    memset(&L, 0, sizeof L);
    L.ctl = S->d_ctl;
    L.cfg = S->d_cfg;
    L.portlut = S->portlut;
    L.in = S->d_in;
    L.out = S->d_out;
    L.scratch = S->d_scratch;
    L.start_seq = start_seq;
    L.idle_ticks = TE_SRV_IDLE_TICKS;
    S->ctl->stop = 0;
    __atomic_store_n(&S->ctl->alive, 1u, __ATOMIC_RELEASE);
    if (te_launch_packet_server(&L, S->stream) != 0) {
        S->ctl->alive = 0;
        te_seterr(t, "packet server launch failed: %s", hipGetErrorString(hipGetLastError()));
        return -1;
    }
    S->running = 1;
    return 0;
}

/* the context's server, running with its current config; NULL: decline (or an error set) */
static te_srv_t *srv_ready(tcpedit_t *t)
{
    te_srv_t *S = t->srv;
    if (!S) {
        S = calloc(1, sizeof *S);
        if (!S)
            return NULL;
        t->srv = S;
        if (hipStreamCreateWithFlags(&S->stream, hipStreamNonBlocking) != hipSuccess ||
            hipHostMalloc((void **)&S->ctl, 4096, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostMalloc((void **)&S->in, TE_SRV_IN, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostMalloc((void **)&S->out, TE_SRV_OUT, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer((void **)&S->d_ctl, S->ctl, 0) != hipSuccess ||
            hipHostGetDevicePointer((void **)&S->d_in, S->in, 0) != hipSuccess ||
            hipHostGetDevicePointer((void **)&S->d_out, S->out, 0) != hipSuccess ||
            hipMalloc((void **)&S->d_scratch, TE_SRV_SCRATCH) != hipSuccess ||
            hipMemset(S->d_scratch, 0, TE_SRV_SCRATCH) != hipSuccess ||
            hipMalloc((void **)&S->d_cfg, sizeof(te_dev_cfg_t)) != hipSuccess) {
            (void)hipGetLastError();
            S->broken = 1;
            return NULL;
        }
        memset(S->ctl, 0, 4096);
        memset(S->in, 0, TE_SRV_IN);
        pthread_mutex_lock(&te_srv_mu);
        int slot = -1;
        for (int i = 0; i < TE_SRV_MAX && slot < 0; i++)
            if (!te_srv_live[i])
                slot = i;
        if (slot >= 0)
            te_srv_live[slot] = S;
        if (!te_srv_atexit_done) {
            atexit(srv_stop_all);
            te_srv_atexit_done = 1;
        }
        pthread_mutex_unlock(&te_srv_mu);
        if (slot < 0) { /* (every slot taken: no server for this context) */
            S->broken = 1;
            return NULL;
        }
    }
    if (S->broken)
        return NULL;
    te_dev_cfg_t want = t->cfg;
    want.skip_soft_errors = 0; /* tcpedit_packet itself never drops */
    const uint16_t *pl = t->cfg.has_portmap ? t->d_portlut : NULL;
    if (S->running && (memcmp(&want, &S->cfg, sizeof want) != 0 || pl != S->portlut || t->portlut != S->hportlut) &&
        srv_stop(S) < 0) {
        S->broken = 1;
        return NULL;
    }
    if (S->running && !__atomic_load_n(&S->ctl->alive, __ATOMIC_ACQUIRE)) { /* it left (idle) */
        hipStreamSynchronize(S->stream);
        S->running = 0;
    }
    if (!S->running) {
        S->cfg = want;
        S->portlut = pl;
        S->hportlut = t->portlut;
        if (hipMemcpyAsync(S->d_cfg, &S->cfg, sizeof S->cfg, hipMemcpyHostToDevice, S->stream) != hipSuccess ||
            hipStreamSynchronize(t->stream) != hipSuccess || hipStreamSynchronize(S->stream) != hipSuccess) {
            te_seterr(t, "packet server setup failed: %s", hipGetErrorString(hipGetLastError()));
            S->broken = 1;
            return NULL;
        }
        if (srv_launch(t, S, S->seq) < 0) {
            S->broken = 1;
            return NULL;
        }
    }
    return S;
}

/* one request; 0 when served, -1 when the server stopped answering */
static int srv_call(tcpedit_t *t, te_srv_t *S)
{
    te_srv_ctl_t *c = S->ctl;
    const uint32_t q = ++S->seq;
    __atomic_store_n(&c->seq, q, __ATOMIC_RELEASE);
    const double t0 = te_now();
    for (unsigned n = 1; __atomic_load_n(&c->done, __ATOMIC_ACQUIRE) != q; n++) {
        __builtin_ia32_pause();
        if ((n & 255) != 0)
            continue;
        if (!__atomic_load_n(&c->alive, __ATOMIC_ACQUIRE)) {
            /* it left (idle timeout) before it saw this request: launch it again */
            if (__atomic_load_n(&c->done, __ATOMIC_ACQUIRE) == q)
                break;
            hipStreamSynchronize(S->stream);
            if (srv_launch(t, S, q - 1) < 0)
                return -1;
        } else if (te_now() - t0 > 5.0 || srv_test_stuck()) {
            te_seterr(t, "packet server did not answer in 5 s");
            srv_stop(S); /* bounded: a kernel that does not leave is left running, unsynced */
            return -1;
        }
    }
    return 0;
}

/* the status byte and output record of one tcpedit_packet edit into the caller's header
 * and buffer (out_img: an image whose record starts at byte 24; out_len: its bytes) */
static int packet_result(tcpedit_t *t, struct pcap_pkthdr *h, unsigned char **pktdata, uint8_t st,
                         const uint8_t *out_img, uint64_t out_len, uint64_t cap)
{
    int rc;
    switch (st & TE_ST_RC_MASK) {
    case TE_ST_RC_ERROR:
        te_seterr(t, "packet %llu: tcpedit error", (unsigned long long)t->pub.runtime.packetnum);
        return TCPEDIT_ERROR;
    case TE_ST_RC_SOFT:
        te_seterr(t, "Packet %llu has no L3+ header or cannot be edited", (unsigned long long)t->pub.runtime.packetnum);
        rc = TCPEDIT_SOFT_ERROR;
        break;
    case TE_ST_RC_WARN:
        rc = TCPEDIT_WARN;
        break;
    default:
        rc = TCPEDIT_OK;
    }
    if (st & TE_ST_WARNED) {
        te_setwarn(t, "packet %llu: checksum not recomputed", (unsigned long long)t->pub.runtime.packetnum);
        fprintf(stderr, "Warning: %s\n", t->pub.runtime.warnstr);
    }
    if (out_len >= 24 + 16) {
        uint32_t oc, ol;
        memcpy(&oc, out_img + 24 + 8, 4);
        memcpy(&ol, out_img + 24 + 12, 4);
        if (oc > 262166u || 40 + (uint64_t)oc > cap) {
            te_seterr(t, "packet %llu: output record of %u bytes", (unsigned long long)t->pub.runtime.packetnum, oc);
            return TCPEDIT_ERROR;
        }
        memcpy(*pktdata, out_img + 40, oc);
        h->caplen = oc;
        h->len = ol;
    } else {
        h->caplen = 0; /* edited down to zero bytes */
    }
    return rc;
}

/* tcpedit_packet through the resident server, or TE_SRV_DECLINED: --fuzz-seed (its state
 * stream), the en10mb dst_modified carry, a record larger than the block's
 * LDS slot, and an edit that reads past caplen take the launch-per-call path */
static int packet_via_server(tcpedit_t *t, struct pcap_pkthdr *h, unsigned char **pktdata, int direction)
{
    if (!srv_enabled() || (t->srv && t->srv->broken))
        return TE_SRV_DECLINED;
    const te_dev_cfg_t *c = &t->cfg;
    if (c->fuzz_seed || (TE_DEC_ETH_ADDR(c->decoder) && c->encoder == TE_ENC_EN10MB && !(c->mac_mask & TE_MASK_DMAC1)) ||
        jnpr_carry_cfg(c)) /* (the Juniper decoder state: the launch path carries it) */
        return TE_SRV_DECLINED;
    const uint32_t caplen = h->caplen;
    uint64_t data = caplen;
    if (c->fixlen == TE_FIXLEN_PAD && h->len > data)
        data = h->len;
    if (data > 262144u || TE_SLOT_BYTES_OF_H(te_slot_head(c), 8u, data) > (uint32_t)TE_SLOT_BYTES)
        return TE_SRV_DECLINED;
    if (te_upload_cfg(t) < 0)
        return TCPEDIT_ERROR;
    te_srv_t *S = srv_ready(t);
    if (!S)
        return TE_SRV_DECLINED; /* (no server could be set up: the launch-per-call path) */
    const uint32_t rh[4] = {(uint32_t)h->ts.tv_sec, (uint32_t)h->ts.tv_usec, caplen, h->len};
    memcpy(S->in + 24, rh, 16);
    memcpy(S->in + 40, *pktdata, caplen);
    memset(S->in + 40 + caplen, 0, 16);
    S->ctl->dir = direction;
    S->ctl->caplen = caplen;
    if (srv_call(t, S) < 0) {
        S->broken = 1;
        return TE_SRV_DECLINED;
    }
    const uint8_t st = (uint8_t)S->ctl->status;
    if (st & TE_ST_UNSUPPORTED)
        return TE_SRV_DECLINED;
    t->pub.runtime.packetnum += S->ctl->packets;
    t->pub.runtime.total_bytes += S->ctl->bytes_out;
    t->pub.runtime.pkts_edited += S->ctl->edited;
    return packet_result(t, h, pktdata, st, S->out, 24 + S->ctl->bytes_out, TE_SRV_OUT);
}

/* tcpedit_packet (tcpedit.c:46-366): one record through the resident server, or through
 * the GPU kernel staged in the context's page-locked one-record batch. */
int tcpedit_packet(tcpedit_t *t, struct pcap_pkthdr **pkthdr, unsigned char **pktdata, tcpr_dir_t direction)
{
    if (!t || !pkthdr || !*pkthdr || !pktdata || !*pktdata)
        return TCPEDIT_ERROR;
    if (te_ensure_cfg(t) < 0)
        return TCPEDIT_ERROR;
    struct pcap_pkthdr *h = *pkthdr;
    const uint32_t caplen = h->caplen;
    if (caplen > 262144u) {
        te_seterr(t, "packet %llu: caplen %u exceeds MAX_SNAPLEN", (unsigned long long)t->pub.runtime.packetnum + 1,
                  caplen);
        return TCPEDIT_ERROR;
    }
    if (direction == TCPR_DIR_S2C && te_check_decoder_cfg(t, 1) < 0)
        return TCPEDIT_ERROR;
    {
        const int r = packet_via_server(t, h, pktdata, (int)direction);
        if (r != TE_SRV_DECLINED)
            return r;
    }
    tcpedit_batch_t *b = one_ready(t);
    if (!b)
        return TCPEDIT_ERROR;
    static const uint8_t fh[24] = {0xd4, 0xc3, 0xb2, 0xa1, 2, 0, 4, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                   0x00, 0x00, 0x04, 0, 1, 0, 0, 0};
    uint8_t *img = b->one_img, *res = b->one_img + TE_ONE_IN;
    const size_t img_len = 24 + 16 + (size_t)caplen;
    memcpy(img, fh, 24);
    {
        const uint32_t lt = (uint32_t)t->dlt; /* the context's DLT (its decoder) */
        memcpy(img + 20, &lt, 4);
    }
    const uint32_t rh[4] = {(uint32_t)h->ts.tv_sec, (uint32_t)h->ts.tv_usec, caplen, h->len};
    memcpy(img + 24, rh, 16);
    memcpy(img + 40, *pktdata, caplen);
    uint8_t saved_skip = t->cfg.skip_soft_errors;
    t->cfg.skip_soft_errors = 0; /* tcpedit_packet itself never drops */
    t->dev_dirty |= saved_skip;
    int rc = TCPEDIT_ERROR;
    /* a different record each call: no launch hint or placement carries over */
    b->pkt_base = t->pub.runtime.packetnum;
    b->launches = 0;
    b->gen_hint_ok = 0;
    b->grow_off = 0;
    b->ran = 0;
    if (index_image(t, b, img, img + 24, img_len) < 0)
        goto out;
    if (b->n_pkts != 1) {
        te_seterr(t, "packet %llu: not a record", (unsigned long long)t->pub.runtime.packetnum + 1);
        goto out;
    }
    HIPCHK(t, hipMemcpyAsync(b->d_in, img, img_len, hipMemcpyHostToDevice, t->stream));
    HIPCHK(t, hipMemcpyAsync(b->d_tiles, b->tiles, sizeof(te_tile_t) * b->n_tiles, hipMemcpyHostToDevice, t->stream));
    HIPCHK(t, hipMemcpyAsync(b->d_pkt_rel, b->pkt_rel, sizeof(uint16_t), hipMemcpyHostToDevice, t->stream));
    b->tcut_ok = 0;
    HIPCHK(t, hipMemsetAsync(b->d_ws, 0, b->ws_bytes, t->stream));
    if (batch_run_dir(t, b, (int)direction) != TCPEDIT_OK)
        goto out;
    {
        /* status byte and the output record in one round trip */
        const uint64_t bound = 24 + b->out_cap < TE_ONE_OUT - 64 ? 24 + b->out_cap : TE_ONE_OUT - 64;
        HIPCHK(t, hipMemcpyAsync(res, b->d_status, 1, hipMemcpyDeviceToHost, t->stream));
        HIPCHK(t, hipMemcpyAsync(res + 64, b->d_out, bound, hipMemcpyDeviceToHost, t->stream));
        HIPCHK(t, hipStreamSynchronize(t->stream));
    }
    if (res[0] & TE_ST_UNSUPPORTED) {
        /* the edit read past caplen: in tcpedit_packet the reference reads the caller's own
           buffer there, so replay over the caller's bytes [0, need) */
        uint32_t ent[4];
        HIPCHK(t, hipMemcpy(ent, b->d_q8, 16, hipMemcpyDeviceToHost));
        const uint32_t need = ent[1] > 262144u ? 262144u : ent[1];
        HIPCHK(t, hipMemcpyAsync(b->d_q8_init, *pktdata, need, hipMemcpyHostToDevice, t->stream));
        if (run_q8(t, b, (int)direction, 1, b->d_q8_init, need, t->stream) < 0)
            goto out;
        const uint64_t bound = 24 + b->out_cap < TE_ONE_OUT - 64 ? 24 + b->out_cap : TE_ONE_OUT - 64;
        HIPCHK(t, hipMemcpyAsync(res, b->d_status, 1, hipMemcpyDeviceToHost, t->stream));
        HIPCHK(t, hipMemcpyAsync(res + 64, b->d_out, bound, hipMemcpyDeviceToHost, t->stream));
        HIPCHK(t, hipStreamSynchronize(t->stream));
    }
    const uint8_t st = res[0];
    if (st & TE_ST_UNSUPPORTED) {
        te_seterr(t, "packet %llu: the edit reads bytes past caplen the replay cannot reproduce (SURVEY Q8)",
                  (unsigned long long)t->pub.runtime.packetnum);
        goto out;
    }
    {
        tcpedit_batch_result_t r;
        tcpedit_batch_result(b, &r);
        rc = packet_result(t, h, pktdata, st, res + 64, r.out_len, 24 + b->out_cap);
    }
out:
fail:
    t->cfg.skip_soft_errors = saved_skip;
    t->dev_dirty |= saved_skip;
    return rc;
}

int tcpedit_close(tcpedit_t **tp)
{
    if (!tp || !*tp)
        return TCPEDIT_ERROR;
    tcpedit_t *t = *tp;
    for (int k = 0; k < OPT__N; k++) {
        free(t->arg[k]);
        for (int i = 0; i < t->nstack[k]; i++)
            free(t->stack[k][i]);
    }
    free(t->portlut);
    srv_free(t);
    for (int w = 0; w < 4; w++) {
        free(t->cspill[w]);
        hipFree(t->d_cspill[w]);
    }
    tcpedit_batch_close(t->one);
    hipFree(t->d_cfg);
    hipFree(t->d_portlut);
    hipFree(t->d_fuzz_words);
    hipFree(t->d_l2word);
    hipFree(t->d_jctx);
    hipFree(t->d_q8_scratch);
    te_pipe_free(t);
    if (t->stream)
        hipStreamDestroy(t->stream);
    free(t);
    *tp = NULL;
    return 0;
}

uint64_t tcpedit_shard_place(int n, const uint64_t *seg_bytes, const int *hard_error, uint64_t *offset,
                             uint64_t *write)
{
    uint64_t pos = 24;
    int failed = 0;
    for (int k = 0; k < n; k++) {
        offset[k] = pos;
        write[k] = failed ? 0 : seg_bytes[k];
        pos += write[k];
        failed |= hard_error[k] != 0;
    }
    return pos;
}

int64_t tcpedit_pcap_shards(const void *pcap, size_t len, int n, uint64_t *off, uint64_t *pkt_base)
{
    const uint8_t *img = pcap;
    if (!img || len < 24 || n < 1 || !off || !pkt_base)
        return -1;
    uint32_t magic;
    memcpy(&magic, img, 4);
    int swapped;
    if (magic == 0xa1b2c3d4u || magic == 0xa1b23c4du)
        swapped = 0;
    else if (magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u)
        swapped = 1;
    else
        return -1;
    /* pass 1: where libpcap's walk ends */
    size_t end = 24;
    uint64_t total = 0;
    while (end + 16 <= len) {
        uint32_t caplen = rd32(img + end + 8, swapped);
        if (caplen > 262144u || end + 16 + caplen > len)
            break;
        end += 16 + caplen;
        total++;
    }
    /* pass 2: cut at the first record boundary at or past k/n of the bytes */
    const uint64_t bytes = end - 24;
    size_t o = 24;
    uint64_t pk = 0;
    off[0] = 24;
    pkt_base[0] = 0;
    for (int k = 1; k < n; k++) {
        const uint64_t target = 24 + bytes * (uint64_t)k / (uint64_t)n;
        while (o < target && o < end) {
            o += 16 + rd32(img + o + 8, swapped);
            pk++;
        }
        off[k] = o;
        pkt_base[k] = pk;
    }
    off[n] = end;
    return (int64_t)total;
}
