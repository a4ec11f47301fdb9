/*
 * te_kernels.h -- the boundary between the C host code and the gfx950 kernels
 * (plain pointers and sizes only).  Shared by tcpedit_kernels.hip and the host.
 */
#ifndef TE_KERNELS_H
#define TE_KERNELS_H

#include <stddef.h>
#include <stdint.h>
#include "te_dev_cfg.h"

#ifdef __cplusplus
extern "C" {
#endif

#define TE_BLOCK 256           /* threads per block = max packets per tile */
#define TE_MAX_PKTS 256
#ifndef TE_SLOT_BYTES
#define TE_SLOT_BYTES 36864    /* LDS slot budget per block (3 blocks / CU) */
#endif
#define TE_HEAD 16             /* least headroom before each record's slot (te_dev_cfg_t.slot_head) */
#define TE_TAIL_BYTES 16       /* zeroed bytes after each packet's data */
#define TE_NO_SCRATCH 0xffffffffffffffffull
#ifndef TE_FK_TILE_BYTES
#define TE_FK_TILE_BYTES 24576 /* tile budget when the fast lane runs */
#endif
#ifndef TE_FK_BLOCK
#define TE_FK_BLOCK 256        /* threads per fast-lane block = max records per fast-lane tile */
#endif
#ifndef TE_WK_TILE_BYTES
#define TE_WK_TILE_BYTES 6144  /* wave-lane tile budget (one wave = one tile of <= 64 records) */
#endif
#ifndef TE_WK_BLOCK
#define TE_WK_BLOCK 256        /* threads per wave-lane block (its waves share only the cfg copy) */
#endif
#define TE_WK_PKTS 64          /* records per wave-lane tile: one per lane */
#define TE_TILE_SOLO 1u        /* te_tile_t.flags: a record too large for a wave-lane image */
#define TE_FAST_BLOCK 1        /* fast-lane kinds: te_fast_tiles (one block per tile) ... */
#define TE_FAST_WAVE 2         /* ... or te_wave_tiles (one wave per tile) */
/* the one record-size change a wave-lane instance (and static placement) carries */
#define TE_SZ_NONE 0
#define TE_SZ_GROW 1           /* --enet-vlan=add: +4 per record */
#define TE_SZ_VDEL 2           /* --enet-vlan=del over tagged records: -4 */
#define TE_SZ_EFCS 3           /* --efcs: -4 */
#define TE_SZ_MTU 4            /* --mtu-trunc: a record longer than the MTU loses its tail */
#define TE_SZ_FUZZ 5           /* --fuzz-seed: a picked record may be cut (DROP / REDUCE) */
/* the wave lane's per-block totals: {records, bytes in, records edited, bytes cut, records
   dropped (not written), soft errors, -, -} */
#define TE_WK_SLOT_WORDS 8
/* option groups of the fast lane: a te_wave_tiles instance compiles in the groups of
   its mask, and te_launch_edit launches the smallest instance covering the config */
#define TE_FF_MAC 1u     /* --enet-dmac / --enet-smac */
#define TE_FF_PORTMAP 2u /* --portmap */
#define TE_FF_RWIP 4u    /* --srcipmap / --dstipmap / --pnat / --endpoints */
#define TE_FF_SEED 8u    /* --seed */
#define TE_FF_ALL 15u
#define TE_FF_HDR 16u    /* --tos / --ttl / --tclass / --flowlabel / --tcp-sequence */
#define TE_FF_INCR 32u   /* no --fixcsum: checksums follow the incremental updates (RFC 1624)
                            unless the packet needs a recompute (needtorecalc, tcpedit.c:338) */
#define TE_FF_ALLX 63u
#define TE_FF_SMALL 64u  /* a mode, not an option group: the lean size-preserving instances cut to
                            5 KiB tiles at 5 blocks/CU, for batches of small records (64 of them, the
                            tile's record cap, fit): te_wave_small(); others take 8 KiB at 3-4 */

/* bytes a record needs in a slot: g = its HBM address mod 16, data = bytes of
 * packet data to materialise (caplen, or max(caplen, len) under --fixlen=pad) */
#define TE_LDS_FRONT 16        /* front pad of the LDS image (funnel reads never go below 0) */

/* contiguous layout: a tile's span (starting g bytes into its 16-byte chunk)
 * fits the LDS image when this holds */
#define TE_CONTIG_FITS_IN(g, span, budget) ((uint32_t)(g) + (uint32_t)(span) + 16u <= (uint32_t)(budget))
#define TE_CONTIG_FITS(g, span) TE_CONTIG_FITS_IN(g, span, TE_SLOT_BYTES)

#define TE_SLOT_BYTES_OF_H(head, g, data) \
    ((((uint32_t)(head) + (uint32_t)(g) + 16u + (uint32_t)(data) + (uint32_t)TE_TAIL_BYTES) + 15u) & ~15u)
#define TE_SLOT_BYTES_OF(g, data) TE_SLOT_BYTES_OF_H(TE_HEAD, g, data)

/* DLT_JUNIPER_ETHER: the decoder state a whole inner decode leaves in the encoder's
 * context (tcpedit_dlt_copy_decoder_state, dlt_utils.c:249-271: addresses, proto, and by
 * the extra pointer the en10mb sub-decoder's VLAN fields), which a later frame whose
 * extensions are not Ethernet -- the reference's TCPEDIT_WARN, jnpr_ether.c:269-272 --
 * is encoded with */
typedef struct {
    uint8_t dstaddr[6], srcaddr[6];
    uint16_t proto;
    uint16_t vlan_tag, vlan_pri, vlan_cfi, vlan_proto;
    uint16_t pad0_;
    uint32_t vlan_offset;
    uint8_t vlan;
    uint8_t pad1_[3];
} te_jstate_t;
/* the context's carried state: TE_JC_NONE no whole decode yet (the encoder's own zeroed
 * extra), TE_JC_VALID the state in .st, TE_JC_UNKNOWN not known here (a shard that starts
 * mid-capture before its carry-in was set: such a frame fails loudly) */
typedef struct {
    te_jstate_t st;
    uint32_t valid;
    uint32_t pad_[3];
} te_jctx_t;
#define TE_JC_NONE 0u
#define TE_JC_VALID 1u
#define TE_JC_UNKNOWN 2u

/* A tile = a run of consecutive pcap records processed by one block. */
typedef struct {
    uint64_t span_off;    /* HBM offset of the first record (its 16-byte header) */
    uint64_t scratch_off; /* TE_NO_SCRATCH, or the HBM scratch slot of a huge record */
    uint32_t first_pkt;   /* index of the first record in this run */
    uint32_t npkt;
    uint32_t span_len;    /* bytes of records in the tile */
    uint32_t flags;       /* TE_TILE_* */
} te_tile_t;

typedef struct {
    const te_dev_cfg_t *cfg;  /* device pointer */
    const te_dev_cfg_t *cfg_host; /* the same config on the host (instance choice, scalar knobs) */
    const uint16_t *portlut;  /* device: 65536-entry first-match port map, or NULL */
    const uint8_t *dirbits;   /* device: tcpprep cache data, or NULL */
    uint64_t dirbits_len;
    uint64_t pkt_base;        /* 0-based packet number of the first record */
    int32_t fixed_dir;        /* >= 0: direction for every record (tcpedit_packet); -1: cache/C2S */
    const uint8_t *in;        /* device: input pcap image */
    const te_tile_t *tiles;   /* device */
    const uint16_t *pkt_rel;  /* device: record offset relative to its tile */
    uint32_t n_tiles;
    uint32_t in_swapped, in_nsec;
    uint8_t *out;             /* device: output pcap image */
    uint64_t out_base;        /* offset of the first output record */
    uint64_t *tile_state;     /* device: n_tiles look-back granules */
    unsigned int *ticket;     /* device */
    uint8_t *status;          /* device: one byte per record */
    uint64_t *counters;       /* device: TE_CNT__N */
    uint64_t *err;            /* device: [0] ~first error record, [1] ~its output offset, [2] timeouts */
    uint8_t *scratch;         /* device: huge-record slots */
    void *zero_region;        /* device range zeroed before each launch */
    uint64_t zero_bytes;
    int grid;                 /* blocks to launch (persistent, tiles taken by ticket) */
    int slot_layout;          /* 1: per-record LDS slots (--enet-vlan=add, --fixlen=pad); 0: contiguous */
    int static_off;           /* 1: no record can change size or be dropped, so every output
                                 record sits at its input offset: no scan, no look-back */
    uint64_t rec0;            /* input offset of the first record (static_off: out = in - rec0 + out_base) */
    int static_grow;          /* 1: every record grows by exactly 4 bytes (VLAN add and no other size
                                 change), so record i (0-based in the launch) sits at its input offset
                                 + 4 i: no scan, no look-back.  A record that breaks this (and is not a
                                 hard error, which truncates the output there) sets *grow_bad */
    int static_shrink;        /* TE_SZ_VDEL / TE_SZ_EFCS: every record shrinks by exactly 4
                                 bytes (a VLAN pop, or --efcs, as the only size change): record i sits
                                 at its input offset - 4 i; a record that breaks it sets *grow_bad */
    uint32_t *grow_bad;       /* device word, zeroed with the error words */
    int static_mtu;           /* --mtu-trunc as the only size change: tile t's output starts at its
                                 input offset - tcut[t], the predicted bytes --mtu-trunc removes from
                                 the records before it (te_mtu_cuts); a tile whose output differs
                                 from the prediction sets *grow_bad */
    const long long *tcut;    /* device: n_tiles + 1 exclusive prefix of the predicted cuts */
    uint32_t mtu;             /* static_mtu: the MTU (cfg.mtu) */
    int wk_small;             /* the batch's tiles were cut for the TE_FF_SMALL instances */
    int static_fz;            /* --fuzz-seed on the wave lane: the launch finds the reaching records
                                 (te_fuzz_reach + the generic reach pass over the tiles it lists),
                                 draws the states, predicts each tile's cut into tcut (written
                                 here, not read) and places tiles by it like static_mtu */
    long long *tcut_raw;      /* static_fz: device scratch, (n_tiles + 63) / 64 + 1 words */
    uint32_t *fz_list;        /* static_fz: device, n_tiles + 1 + n_pkts words (the reach list, its
                                 count, a word per record for the cut prediction) */
    /* fast lane (static_off configs the register-resident lane carries): te_fast_tiles edits
       every tile it can, appends the rest to tile_list, and the generic kernel then redoes
       only the listed tiles */
    int fast;
    int fast_kind;            /* TE_FAST_BLOCK or TE_FAST_WAVE (how the tiles were cut) */
    uint64_t *slots;          /* device: wave lane's per-block totals (TE_WK_SLOT_WORDS words); the
                                 host adds them to this launch's counters */
    int skip_generic;         /* wave lane: leave out the generic pass (no tile will be listed) */
    int generic_only;         /* run only the generic pass over the tiles the last fast launch listed */
    int out_fgrid;            /* set by te_launch_edit: blocks of the fast-lane launch (slots written) */
    int fast_v6;              /* IPv6 packets may take the fast lane (no non-octet v6 CIDR maps) */
    int stream;               /* wave lane: nontemporal loads/stores (the batch outgrows the MALL) */
    uint32_t *tile_list;      /* device: n_tiles entries */
    uint32_t *list_cnt;       /* device: 2 counts; launch parity p appends to [p] and zeroes [p^1] */
    uint32_t parity;
    uint64_t *counters_next;  /* fast lane: the other parity's counter set, zeroed for the next launch */
    uint64_t *ws_zero;        /* device: 4 words (err, ticket) the fast kernel zeroes */
    void *ev_k0, *ev_k1;      /* optional hipEvent_t pair recorded around the dominant edit kernel */
    /* --fuzz-seed (generic lane only): a reach pass, then per-record RNG states, then the edit */
    uint32_t *fuzz_states;    /* device: n_pkts words, or NULL (no fuzzing) */
    uint32_t *fuzz_blk;       /* device: a word per 1024 records */
    uint32_t *fuzz_words;     /* device: [0] the context's running RNG state, [1] this launch's start,
                                 [2] records of the launch that reached the fuzz step */
    uint32_t n_pkts;          /* records in the launch */
    int fuzz_probe_only;      /* count the reaching records (words[2]) and stop: no edit, no state change */
    int q18_only;             /* --fuzz-seed with the Q18 carry: the states (from the running start, which
                                 stays) and the carry's mark run and scan, then stop: no edit */
    /* stale static-buffer reads: the edit lists such written records here as
       {record, bytes needed, output offset lo, hi}; te_launch_q8 replays them */
    void *q8_list;            /* device: q8_cap x 16 bytes, or NULL */
    uint32_t q8_cap;
    void *q8_scratch;         /* device: q8_threads x te_q8_slot_bytes() */
    uint32_t q8_threads;      /* a multiple of 64 */
    int q8_file_start;        /* the launch's first record is the capture's first (buffer starts zeroed) */
    const uint8_t *q8_init;   /* device: the initial buffer instead of zeros (tcpedit_packet), or NULL */
    uint32_t q8_init_len;
    /* the records just before the launch's first (the previous pipeline chunk's or shard's
       last ones): the replay may walk back into them (records -q8_npre .. -1) */
    const uint8_t *q8_pre;    /* device: their bytes (whole records, the launch's format) */
    const uint64_t *q8_pre_off; /* device: q8_npre offsets into q8_pre */
    uint32_t q8_npre;
    int q8_pre_file_start;    /* the first of them is the capture's first record */
    /* SURVEY Q18 (a Linux cooked decoder into the en10mb encoder without --enet-dmac): the
       dst_modified carry.  NULL: none (every record's value is its own or false) */
    uint64_t *l2carry;        /* device: n_pkts + 1 scan results */
    uint64_t *l2carry_keys;   /* device: n_pkts + 1 keys */
    uint32_t *l2carry_word;   /* device: the context's value after its last launch */
    void *l2carry_tmp;        /* device: te_l2carry_temp_bytes(n_pkts) of scan scratch */
    size_t l2carry_tmp_bytes;
    /* DLT_JUNIPER_ETHER into an encoder that reads the decoder state: each record's last
       whole inner decode before it (te_jnpr_mark + an inclusive max scan: jscan[j] = i + 1
       for record i, 0 = none in the launch, then *jctx).  NULL: none */
    uint64_t *jscan;          /* device: n_pkts + 1 scan results */
    uint64_t *jkeys;          /* device: n_pkts + 1 keys */
    te_jstate_t *jstates;     /* device: n_pkts + 1 states (entry i + 1: record i's) */
    te_jctx_t *jctx;          /* device: the context's carried state */
    void *jtmp;               /* device: te_l2carry_temp_bytes(n_pkts) of scan scratch */
    size_t jtmp_bytes;
    int any_dec;              /* a non-Ethernet decoder or a non-encoding / pppserial encoder: the
                                 generic kernel's instance that carries them */
    /* window mode (te_launch_edit with win set): the wave lane finds the records itself, no
       tiles or record index -- byte windows of the image from win_base, the first record at
       win_entry (or *win_entry_ptr - win_entry_sub on the device), records starting at
       win_limit on not the image's; te_win_check then checks the chain across windows */
    int win;
    uint64_t win_len, win_entry, win_entry_sub, win_base, win_limit;
    const uint64_t *win_entry_ptr;
    uint32_t nwin;
    uint64_t *w_entry, *w_exit;  /* device: nwin words each */
    uint32_t *w_flags;           /* device: nwin words */
    uint32_t *win_bad;           /* device word, zeroed by the launch: bit 0 the chain missed or
                                    stopped, bit 1 a record left to the exact path */
    uint64_t *win_tot;           /* device: [0] the chain's end (image offset), zeroed by the launch */
    /* the window-mode pipeline's per-chunk steps, in the check's launch: the call's device
       accumulator {packets, bytes, edited, verdict} (or NULL), and the previous chunk's output
       image whose bytes before this chunk's first record are copied in (or NULL; a first
       record past win_head_max is no chain's: nothing copied) */
    uint64_t *win_acc;
    const uint8_t *win_prev_out;
    uint64_t win_head_max;
    uint64_t win_org;            /* image offset of the chunk's first file byte (0: 24) */
} te_launch_t;
/* bytes a window of the window mode owns */
uint32_t te_win_bytes(void);

/* tcpedit_packet's resident server (te_packet_server, one block): a control block in
 * host-mapped fine-grained memory.  The host writes the record at byte 24 of the mapped
 * input image, the request words dir and caplen, then seq (release); the kernel polls the
 * first 16 bytes {seq, stop, dir, caplen} with one read -- a new seq arrives together with
 * the request it publishes (x86 keeps the host's stores in order), so a request costs one
 * PCIe read round trip, not two -- edits the record into the mapped output image (record
 * at byte 24), writes the response words and stores done = seq (release).  It leaves when
 * stop is set or after idle_ticks of the 100 MHz real-time clock without a request,
 * storing alive = 0.  (The server edits with a fixed direction: no cache lookup, so it
 * needs no packet number.) */
typedef struct {
    uint32_t seq;       /* host: the request number */
    uint32_t stop;      /* host: 1 = leave now */
    int32_t dir;        /* request: the direction (tcpedit_packet's argument) */
    uint32_t caplen;    /* request: the record's caplen (its 16-byte header is in the image) */
    uint32_t done;      /* device: the last request served */
    uint32_t alive;     /* host: 1 before a launch; device: 0 when it leaves */
    /* response */
    uint32_t status;    /* the record's TE_ST_* byte */
    uint32_t pad_;
    uint64_t bytes_out, packets, edited; /* the record's counters (TE_CNT_*) */
} te_srv_ctl_t;

typedef struct {
    te_srv_ctl_t *ctl;         /* device address of the mapped control block */
    const te_dev_cfg_t *cfg;   /* device: the server's config (copied to LDS at launch) */
    const uint16_t *portlut;   /* device, or NULL */
    const uint8_t *in;         /* device address of the mapped input image */
    uint8_t *out;              /* device address of the mapped output image */
    uint8_t *scratch;          /* device: TE_SRV_SCRATCH bytes (status, counters, error words) */
    uint32_t start_seq;        /* the last request served before this launch */
    uint64_t idle_ticks;       /* leave after this long without a request (100 MHz ticks) */
} te_srv_launch_t;
#define TE_SRV_SCRATCH 1024

/* scan scratch the dst_modified carry needs for a launch of n_pkts records */
size_t te_l2carry_temp_bytes(uint32_t n_pkts);

/* blocks of te_fast_tiles / te_wave_tiles resident on the current device */
int te_fast_grid(void);
int te_wave_grid(void);
uint32_t te_wave_waves(const te_dev_cfg_t *c, int sz, int small);

#ifdef __HIP_PLATFORM_AMD__
int te_launch_edit(te_launch_t *L, hipStream_t stream);
int te_launch_q8(te_launch_t *L, hipStream_t stream);
int te_launch_l2carry(te_launch_t *L, hipStream_t stream);
/* the Juniper state scan alone, and the state the launch leaves in *out (a shard's carry-out) */
int te_launch_jnpr(te_launch_t *L, te_jctx_t *out, hipStream_t stream);

int te_launch_packet_server(const te_srv_launch_t *S, hipStream_t stream);
/* --mtu-trunc placement: pre = the exclusive prefix (n_tiles + 1 entries) of the bytes each
   tile's records lose to the truncation, predicted from each record's header and type field
   (len > mtu + l2len: caplen becomes l2len + mtu); bsum: (n_tiles + 63) / 64 + 1 entries of
   scratch (per-64-tile sums) */
int te_mtu_cuts(const uint8_t *in, const te_tile_t *tiles, const uint16_t *pkt_rel, uint32_t n_tiles, uint32_t mtu,
                long long *bsum, long long *pre, hipStream_t stream);
#endif
uint64_t te_q8_slot_bytes(void);
/* tile budget of the wave-lane instance the config launches (sz: TE_SZ_*) */
uint32_t te_wave_tile_bytes(const te_dev_cfg_t *c, int sz, int small);

#ifdef __cplusplus
}
#endif
#endif
