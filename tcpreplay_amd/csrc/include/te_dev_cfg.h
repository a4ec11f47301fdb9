/*
 * te_dev_cfg.h -- the per-run constant tables the host derives once from the
 * tcpedit option surface (tcpedit_post_args, src/tcpedit/parse_args.c:34-254,
 * and dlt_en10mb_parse_opts, src/tcpedit/plugins/dlt_en10mb/en10mb.c:226-396)
 * and hands to the gfx950 kernels.  Plain C POD: included by the C host code
 * and by the HIP kernels.  Lists the reference keeps as linked lists (CIDR maps,
 * --enet-subsmac) become bounded arrays; the port map becomes a 64 K-entry
 * first-match lookup table held separately in HBM.
 */
#ifndef TE_DEV_CFG_H
#define TE_DEV_CFG_H

#include <stdint.h>

#define TE_MAX_CIDRMAP 16
#define TE_MAX_SUBS 32
#define TE_MAX_PM 64

/* tcpr_cidr_t (src/common/cidr.h) */
typedef struct {
    int32_t family;  /* 4 or 6 */
    int32_t masklen;
    uint32_t network; /* network byte order as inet_aton stores it */
    uint8_t network6[16];
} te_cidr_t;

/* tcpr_cidrmap_t: one from->to pair */
typedef struct {
    te_cidr_t from, to;
} te_cidrmap_t;

enum { TE_TTL_OFF = 0, TE_TTL_SET, TE_TTL_ADD, TE_TTL_SUB };       /* tcpedit_types.h:38-43 */
enum { TE_FIXLEN_OFF = 0, TE_FIXLEN_PAD, TE_FIXLEN_TRUNC, TE_FIXLEN_DEL };
enum { TE_VLAN_OFF = 0, TE_VLAN_DEL, TE_VLAN_ADD };
/* encoders: en10mb, user, hdlc; NOENC = linuxsll/linuxsll2/raw/null/loop, whose encode
   always fails (linuxsll.c:201-208, ...); PPP = pppserial, whose encode is a no-op
   (pppserial.c:239-251) */
enum { TE_ENC_EN10MB = 0, TE_ENC_USER, TE_ENC_HDLC, TE_ENC_NOENC, TE_ENC_PPP };
/* decoders (tcpedit_dlt_init by the input DLT; NULL and LOOP share dlt_null's functions) */
enum { TE_DEC_EN10MB = 0, TE_DEC_SLL, TE_DEC_SLL2, TE_DEC_RAW, TE_DEC_NULL, TE_DEC_PPP, TE_DEC_CHDLC,
       TE_DEC_JNPR, TE_DEC_80211, TE_DEC_RADIOTAP };
/* decoders whose plugin_l2addr_type is ETHERNET besides en10mb: the en10mb encoder takes
   their decoded addresses and sets dst_modified from them */
#define TE_DEC_ETH_ADDR(d) ((d) == TE_DEC_SLL || (d) == TE_DEC_SLL2 || (d) == TE_DEC_JNPR || (d) == TE_DEC_80211 || \
                            (d) == TE_DEC_RADIOTAP)
enum { TE_FUZZ_OFF = 0, TE_FUZZ_PROBE, TE_FUZZ_APPLY }; /* the generic kernel's fuzz passes */
#define TE_USER_L2MAX 256 /* USER_L2MAXLEN (255, user_types.h:37), rounded */                  /* en10mb_types.h:50-54 */
enum { TE_MASK_SMAC1 = 1, TE_MASK_SMAC2 = 2, TE_MASK_DMAC1 = 4, TE_MASK_DMAC2 = 8 };
enum { TE_DIR_NOSEND = 0, TE_DIR_C2S = 1, TE_DIR_S2C = 2 };          /* cache.h:77-80 */

typedef struct {
    /* tcpedit_t (tcpedit_types.h:91-153) */
    uint8_t skip_broadcast, rewrite_ip, fixcsum, efcs;
    uint8_t mtu_truncate, fixhdrlen, l2_skip_broadcast, skip_soft_errors;
    int32_t fixlen;
    int32_t ttl_mode;
    uint32_t ttl_value;
    int32_t tos, flowlabel, tclass, mtu;
    uint32_t tcp_sequence_enable, tcp_sequence_adjust;
    uint32_t seed;
    int32_t has_portmap;
    int32_t n_cidrmap1, n_cidrmap2, n_srcipmap, n_dstipmap;
    te_cidrmap_t cidrmap1[TE_MAX_CIDRMAP];
    te_cidrmap_t cidrmap2[TE_MAX_CIDRMAP];
    te_cidrmap_t srcipmap[TE_MAX_CIDRMAP];
    te_cidrmap_t dstipmap[TE_MAX_CIDRMAP];
    /* en10mb_config_t (en10mb_types.h:60-92) */
    uint8_t intf1_dmac[6], intf1_smac[6], intf2_dmac[6], intf2_smac[6];
    int32_t n_subs;
    uint8_t subs[TE_MAX_SUBS][12]; /* target[6], rewrite[6] */
    uint32_t random_set;
    int32_t random_keep;
    uint8_t random_mask[8];
    int32_t mac_mask;
    int32_t vlan;
    uint32_t vlan_tag; /* 65535 = unset */
    uint32_t vlan_pri; /* 255 = unset */
    uint32_t vlan_cfi; /* 255 = unset */
    uint32_t vlan_proto;
    /* the port map's non-identity LUT entries (index and value are the raw little-endian
     * u16 of the network-order port), so the wave lane looks ports up in LDS; -1 when
     * there are more than TE_MAX_PM of them (then the 64 Ki-entry LUT in HBM) */
    int32_t n_pm;
    uint16_t pm_from[TE_MAX_PM];
    uint16_t pm_to[TE_MAX_PM];
    /* the encoder (tcpedit_dlt_post_args, dlt_plugins.c:168-204) and its options:
     * user_config_t (dlt_user/user_types.h:46-55), hdlc_config_t (dlt_hdlc/hdlc_types.h) */
    int32_t encoder;        /* TE_ENC_* */
    int32_t out_linktype;   /* tcpedit_dlt_output_dlt (dlt_plugins.c:268-283) */
    int32_t user_length;    /* --user-dlink bytes, -1 = none */
    uint32_t hdlc_address, hdlc_control; /* 65535 = unset */
    uint8_t user_l2client[TE_USER_L2MAX];
    uint8_t user_l2server[TE_USER_L2MAX];
    /* --fuzz-seed (fuzzing.c:12-20): the mixed seed (0 = off) and --fuzz-factor */
    uint32_t fuzz_seed, fuzz_factor;
    /* the decoder (TE_DEC_*) and whether the launch hands each record the en10mb encoder's
       dst_modified carried from the last C2S record (a Linux cooked decoder
       into the en10mb encoder without --enet-dmac; te_l2carry_mark + a max scan) */
    int32_t decoder;
    uint32_t l2carry;
    /* CIDR maps longer than TE_MAX_CIDRMAP pairs (the reference's lists are unbounded,
       cidr.c:290-418): device addresses of entries TE_MAX_CIDRMAP.. of cidrmap1, cidrmap2,
       srcipmap and dstipmap (0: none), read through TE_CMAP */
    uint64_t cidr_spill[4];
    /* bytes of headroom before each record's slot on the generic lane (slot layouts): room
       for the most the record's L2 header can grow -- a VLAN push, a longer encoder header,
       twice over for a fuzzed record, which is decoded and encoded again (tcpedit.c:89,
       250-258) -- a multiple of 16, at least TE_HEAD */
    uint32_t slot_head;
    uint32_t pad_;
} te_dev_cfg_t;

/* entry i of CIDR map w (0 cidrmap1, 1 cidrmap2, 2 srcipmap, 3 dstipmap): the first
   TE_MAX_CIDRMAP inline, the rest in the spill list */
#define TE_CMAP_INLINE(c, w, i) \
    ((w) == 0 ? (c).cidrmap1[i] : (w) == 1 ? (c).cidrmap2[i] : (w) == 2 ? (c).srcipmap[i] : (c).dstipmap[i])
#define TE_CMAP(c, w, i)                                                                                   \
    ((i) < TE_MAX_CIDRMAP ? TE_CMAP_INLINE(c, w, i)                                                        \
                          : ((const te_cidrmap_t *)(uintptr_t)(c).cidr_spill[w])[(i) - TE_MAX_CIDRMAP])

/* Per-packet status byte written by the device (one per input record). */
enum {
    TE_ST_RC_MASK = 0x03, /* low 2 bits: 0 OK, 1 WARN, 2 SOFT_ERROR, 3 ERROR */
    TE_ST_RC_OK = 0,
    TE_ST_RC_WARN = 1,
    TE_ST_RC_SOFT = 2,
    TE_ST_RC_ERROR = 3,
    TE_ST_DROPPED = 0x04,     /* soft error suppressed by --skip-soft-errors */
    TE_ST_NOSEND = 0x08,      /* cache said NOSEND: written unedited */
    TE_ST_UNSUPPORTED = 0x10, /* output depends on stale static-buffer bytes: fixed by
                                 te_q8_replay, or (still set after it) not reproducible */
    TE_ST_WARNED = 0x20,      /* a checksum warning was emitted (tcpedit.c:351-353) */
    TE_ST_ZEROCAP = 0x40,     /* caplen 0 after editing: not written (tcprewrite.c:367) */
};

/* Counters reduced across tiles (and across GPUs by one RCCL all-reduce). */
enum {
    TE_CNT_PACKETS = 0,
    TE_CNT_BYTES_IN,
    TE_CNT_BYTES_OUT,
    TE_CNT_WRITTEN,
    TE_CNT_EDITED,
    TE_CNT_SOFT,
    TE_CNT_WARN,
    TE_CNT_ERROR,
    TE_CNT_UNSUPPORTED,   /* written records whose edit read stale static-buffer bytes (Q8) */
    TE_CNT_Q8_FAILED,     /* ... that te_q8_replay could not reproduce (the batch fails) */
    TE_CNT__N
};

#endif
