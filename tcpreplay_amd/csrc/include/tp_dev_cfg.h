/*
 * tp_dev_cfg.h -- tcpprep's per-packet classification options as the gfx950
 * kernel reads them (tcpprep_opt_t, src/tcpprep_opts.h, reduced to the
 * per-packet modes).  Shared by the C host (tp_api.c) and the kernel.
 */
#ifndef TP_DEV_CFG_H
#define TP_DEV_CFG_H
#include <stdint.h>
#include "te_dev_cfg.h"

#define TP_MAXC 64

enum { TP_MODE_CIDR = 1, TP_MODE_MAC = 2, TP_MODE_PORT = 3, TP_MODE_AUTO = 4, TP_MODE_REGEX = 5 };
/* the auto modes (tcpprep.c:480-587) */
enum { TP_AUTO_BRIDGE = 1, TP_AUTO_CLIENT, TP_AUTO_SERVER, TP_AUTO_FIRST, TP_AUTO_ROUTER };
/* xX.h:34-41 */
enum { TP_XX_SOURCE = 1, TP_XX_DEST = 2, TP_XX_BOTH = 4, TP_XX_EITHER = 8, TP_XX_PACKET = 16, TP_XX_EXCLUDE = 128 };

/* --regex as a DFA over the characters inet_ntop prints (tp_regex.c): symbols '0'-'9',
   'a'-'f', '.', ':' (0-17), the string start and end (18, 19); state 0 is the absorbing
   match state */
#define TP_NSYM 20
#define TP_SYM_BOS 18
#define TP_SYM_EOS 19
#define TP_DFA_MAX 255
typedef struct {
    uint8_t next[TP_DFA_MAX][TP_NSYM];
    int32_t start, nstates;
} tp_dfa_t;

typedef struct {
    int32_t mode, reverse, nonip, mac_first_empty;
    int32_t ncidr, nmac, xx_mode, nxx_cidr;
    int32_t nlist, automode;
    int32_t dlt, pad_;           /* the capture's link type (get_l2len_protocol's datalink) */
    double ratio;                /* --ratio (default 2.0) */
    uint64_t pkt_base;           /* records before this capture (a shard's place in the job) */
    te_cidr_t cidr[TP_MAXC];     /* -c list (check_ip_cidr: empty list matches all) */
    te_cidr_t xx_cidr[TP_MAXC];  /* -x/-X S:/D:/B:/E: list */
    uint8_t mac[TP_MAXC][8];     /* -e list, as macinstring's mac2hex leaves each token */
    uint64_t lmin[TP_MAXC], lmax[TP_MAXC]; /* -x/-X P: list */
    uint32_t svc_tcp[2048], svc_udp[2048]; /* services bitmaps (tcpprep_api.c:50-53: ports 0-1023) */
    tp_dfa_t dfa;                /* --regex */
} tp_dev_cfg_t;

/* the auto modes' host table in HBM (tree.c's RB tree): open addressing on exact
   64-bit keys -- IPv4: 1<<63 | address; IPv6: one key for every address, as
   tree_comp compares an IPv6 address with itself (tree.c:618-621) */
typedef struct {
    uint64_t *slots;    /* 2 words per slot, one 16-byte pair: the key (0 = empty) and the node's
                           counts (server << 32 | client), or in first mode ~min over sightings
                           of 2 * entry + (0 source | 1 destination) */
    uint32_t *slot;     /* per entry: its source's slot, or ~0 for a non-IP record */
    uint64_t mask;      /* capacity - 1 (power of two, >= 2x the insertions) */
    uint64_t *err;      /* min entry index whose packet2tree hit len_error (init ~0) */
} tp_tree_t;

#ifdef __cplusplus
extern "C" {
#endif
/* auto modes, first pass: build the host table (tree); then tp_launch_classify */
int tp_launch_tree(const uint8_t *img, const uint64_t *off, const uint32_t *caplen, uint64_t n_entries,
                   const tp_dev_cfg_t *cfg, int automode, uint64_t base, tp_tree_t tree, void *stream);
/* sharded auto modes: every node's value from the merged table (keys sorted, unique) */
int tp_launch_tree_merged(tp_tree_t tree, uint64_t capacity, const uint64_t *keys, const uint64_t *vals, uint64_t n,
                          void *stream);
/* classify n_entries records (data at img + off[j], caplen[j], record number
   pktnum[j] or j + 1) into packed 2-bit cache entries out[(n + 3) / 4] */
int tp_launch_classify(const uint8_t *img, const uint64_t *off, const uint32_t *caplen, const uint32_t *pktnum,
                       uint64_t n_entries, const tp_dev_cfg_t *cfg, const tp_tree_t *tree, uint8_t *out,
                       void *stream);
#ifdef __cplusplus
}
#endif
#endif
