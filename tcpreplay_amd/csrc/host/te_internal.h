/*
 * te_internal.h -- host-side state of a tcpedit context (the counterpart of
 * the reference's tcpedit_t, tcpedit_types.h:91-153, whose per-packet half now
 * lives in te_dev_cfg_t on the GPU).
 */
#ifndef TE_INTERNAL_H
#define TE_INTERNAL_H

#ifndef __HIP_PLATFORM_AMD__
#define __HIP_PLATFORM_AMD__
#endif
#include <hip/hip_runtime_api.h>
#include <stdbool.h>
#include <stdint.h>
#include "../../../include/tcpedit.h"
#include "te_dev_cfg.h"
#include "te_kernels.h"

#define TE_ERRSTR_LEN 1024
#define TE_MAX_STACK 256

/* option ids of the tcpedit + DLT option surface */
enum {
    OPT_PORTMAP, OPT_SEED, OPT_PNAT, OPT_SRCIPMAP, OPT_DSTIPMAP, OPT_ENDPOINTS, OPT_TCP_SEQUENCE, OPT_SKIPBROADCAST,
    OPT_FIXCSUM, OPT_FIXHDRLEN, OPT_MTU, OPT_MTU_TRUNC, OPT_EFCS, OPT_TTL, OPT_TOS, OPT_TCLASS, OPT_FLOWLABEL,
    OPT_FIXLEN, OPT_FUZZ_SEED, OPT_FUZZ_FACTOR, OPT_DLT, OPT_SKIPL2BROADCAST, OPT_ENET_DMAC, OPT_ENET_SMAC,
    OPT_ENET_SUBSMAC, OPT_ENET_MAC_SEED, OPT_ENET_MAC_SEED_KEEP_BYTES, OPT_ENET_VLAN, OPT_ENET_VLAN_TAG,
    OPT_ENET_VLAN_CFI, OPT_ENET_VLAN_PRI, OPT_ENET_VLAN_PROTO, OPT_SKIP_SOFT_ERRORS, OPT_USER_DLT, OPT_USER_DLINK,
    OPT_HDLC_CONTROL, OPT_HDLC_ADDRESS, OPT__N
};

typedef struct {
    const char *name;
    char shortopt;
    int has_arg;
    int max;       /* AutoOpts `max` (stacked options allow many) */
    int stacked;
} te_optdef_t;

extern const te_optdef_t te_optdefs[OPT__N];

/* the DLT plugin handle (plugins_types.h:100-131 tcpeditdlt_s, reduced to what the
 * exported accessors answer: the selected decoder and encoder) */
struct tcpeditdlt_s {
    tcpedit_t *tcpedit;
    int decoder_dlt;   /* input DLT */
    int encoder_dlt;   /* the encoder plugin's DLT (DLT_USER0 for user) */
};

enum { TE_SRC_STORE = 1, TE_SRC_SETTERS = 2 }; /* where the options came from */

struct tcpedit_s {
    tcpedit_ref_t pub;            /* the reference's tcpedit_t layout, kept in step (tcpedit.h) */
    struct tcpeditdlt_s dltc;     /* pub.dlt_ctx points here */
    int dlt;                      /* input DLT */
    int device;
    int opt_src;                  /* TE_SRC_* bits: the option store was filled / a setter ran */
    int encoder_set;              /* an encoder was selected by tcpedit_set_encoder_dltplugin_* */
    /* option store (AutoOpts stand-in) */
    int have[OPT__N];
    char *arg[OPT__N];
    char *stack[OPT__N][TE_MAX_STACK];
    int nstack[OPT__N];
    /* derived per-run tables */
    te_dev_cfg_t cfg;
    uint16_t *portlut;            /* host copy, 65536 entries, or NULL */
    te_cidrmap_t *cspill[4];      /* CIDR map entries past TE_MAX_CIDRMAP (cfg.cidr_spill order) */
    te_cidrmap_t *d_cspill[4];    /* ... on the device (uploaded with the config) */
    int32_t d_cspill_n[4];
    uint32_t fuzz_seed, fuzz_factor;
    int post_args_done;
    /* --fuzz-seed state seeding (fuzzing_init): the device word was seeded ... */
    int fz_seeded;                /* ... since the last derivation ... */
    uint64_t fz_gen;              /* ... under this fuzzing_init generation */
    /* device side */
    hipStream_t stream;
    te_dev_cfg_t *d_cfg;
    uint16_t *d_portlut;
    uint32_t *d_fuzz_words;       /* --fuzz-seed: [0] the running RNG state (te_launch_t.fuzz_words) */
    uint8_t *d_q8_scratch;        /* te_q8_replay's emulated static buffers (allocated on first use) */
    uint32_t *d_l2word;           /* the en10mb encoder's dst_modified after the last launch */
    te_jctx_t *d_jctx;            /* DLT_JUNIPER_ETHER: the decoder state the last whole inner decode left */
    int dev_dirty;                /* cfg changed since last upload */
    uint32_t cfg_gen;             /* uploads so far (batches key cached launch hints to it) */
    tcpedit_batch_t *one;         /* reusable one-record batch for tcpedit_packet() */
    struct te_pipe_s *pipe;       /* tcpedit_rewrite_pcap_pipelined's slots and streams (kept) */
    struct te_srv_s *srv;         /* tcpedit_packet's resident server (te_packet_server), or NULL */
    int pipe_err;                 /* that call hit a hard error */
    uint64_t pipe_fallbacks;      /* pipelined calls whose window mode missed (redone exactly) */
};

#define TE_ERR(t) ((t)->pub.runtime.errstr)
#define TE_WARN(t) ((t)->pub.runtime.warnstr)

void te_seterr(tcpedit_t *t, const char *fmt, ...);
void te_setwarn(tcpedit_t *t, const char *fmt, ...);
uint32_t te_tcpr_random(uint32_t *seed);
int te_derive_cfg(tcpedit_t *t); /* tcpedit_post_args body */
int te_upload_cfg(tcpedit_t *t);
int te_ensure_cfg(tcpedit_t *t);  /* derive (or finalize setter values) once before a run */
void te_cfg_defaults(te_dev_cfg_t *c, int dlt);
int te_decoder_of(int dlt);
int te_default_encoder(int dec);
int te_decoder_l2len(int dec);
uint32_t te_slot_head(const te_dev_cfg_t *c);
int te_batch_set_dirbits_dev(tcpedit_batch_t *b, uint8_t *d_bits, uint64_t len);
int te_check_decoder_cfg(tcpedit_t *t, int s2c);
void te_sync_pub(tcpedit_t *t);   /* mirror the derived values into the reference-layout head */
int te_autoopts_import(tcpedit_t *t); /* 1 imported, 0 no descriptor, -1 error (te_autoopts.c) */
extern uint64_t te_fuzz_init_gen; /* fuzzing_init calls so far, and their values */
extern uint32_t te_fuzz_init_seed, te_fuzz_init_factor;
typedef struct te_pipe_s te_pipe_t;
typedef struct te_srv_s te_srv_t;
void te_pipe_free(tcpedit_t *t);

/* te_pcapng.c: a pcapng image as libpcap's reader delivers it (classic pcap, microseconds) */
int te_is_pcapng(const uint8_t *img, size_t len);
int te_pcapng_to_pcap(const uint8_t *in, size_t len, uint8_t **out_img, size_t *out_len, char *err, size_t errlen);
#endif
