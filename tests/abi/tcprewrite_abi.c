/*
 * tcprewrite_abi.c -- the reference tcprewrite's call sequence against
 * include/tcpedit.h, as a relinked tcprewrite would make it (test program).
 *
 * main() follows src/tcprewrite.c:61-183 call for call:
 *   optionProcess(&tcprewriteOptions)  :72   (here: a small parser filling the same
 *                                            AutoOpts descriptors libopts fills)
 *   post_args -> pcap_open_offline     :87,244-247
 *   tcpedit_init(&tcpedit, dlt)        :80
 *   tcpedit_post_args(tcpedit)         :87   (no other option source: the library
 *                                            must read tcprewriteOptions itself)
 *   tcpedit_validate(tcpedit)          :96
 *   fuzzing_init(tcpedit->fuzz_seed, tcpedit->fuzz_factor)  :103 (fields read
 *                                            straight out of the context)
 *   tcpedit_get_output_dlt -> pcap_open_dead(dlt, 65535) + pcap_dump_open  :124,147
 *   rewrite_packets                    :156 -> :260-373 (static MAXPACKET buffer,
 *                                            check_cache, tcpedit_packet per record,
 *                                            --skip-soft-errors, pcap_dump)
 *   tcpedit_close                      :170
 * and exits the way tcprewrite does on each error.
 *
 * The tOptions / tOptDesc / tArgList declarations restate libopts' layout
 * (libopts/autoopts/options.h:194-201, 519-579, 603-680) -- a tool compiled with the
 * real header lays its option set out the same way (tests/golden/autoopts_layout.json
 * pins the offsets).
 *
 * `--print-layout` prints this program's offsets; `--check-options` stops after
 * tcpedit_post_args and prints the derived table's bytes (hex) for comparison with the
 * same options fed through tcpedit_parse_args (CPU-only, no device is touched).
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tcpedit.h"

/* ---- libopts layout (options.h) ------------------------------------------- */
typedef struct {
    uint16_t optIndex, optValue, optActualIndex, optActualValue;
    uint16_t optEquivIndex, optMinCt, optMaxCt, optOccCt;
    uint32_t fOptState;
    uint32_t optUsage;
    union {
        const char *argString;
        long argInt;
    } optArg;
    void *optCookie;
    const int *pOptMust, *pOptCant;
    void (*pOptProc)(void *, void *);
    const char *pzText, *pz_NAME, *pz_Name, *pz_DisableName, *pz_DisablePfx;
} tOptDesc;

typedef struct {
    int useCt;
    int allocCt;
    const char *apzArgs[6];
} tArgList;

typedef struct {
    int structVersion;
    unsigned int origArgCt;
    char **origArgVect;
    uint32_t fOptSet;
    unsigned int curOptIdx;
    char *pzCurOpt;
    const char *pzProgPath, *pzProgName, *pzPROGNAME, *pzRcName, *pzCopyright, *pzCopyNotice, *pzFullVersion;
    const char *const *papzHomeList;
    const char *pzUsageTitle, *pzExplain, *pzDetail;
    tOptDesc *pOptDesc;
    const char *pzBugAddr;
    void *pExtensions, *pSavedState, *pUsageProc, *pTransProc;
    struct {
        uint16_t more_help, save_opts, number_option, default_opt;
    } specOptIdx;
    int optCt;
    int presetOptCt;
} tOptions;

#define OPTST_SET 0x0000001U
#define OPTST_STACKED 0x0000400U
#define OPTST_ARG_TYPE_SHIFT 12
enum { ARG_NONE = 0, ARG_STRING = 1, ARG_NUMBER = 5 };

/* tcprewrite's option set: its own options (tcprewrite_opts.def:108-311) and the
 * tcpedit + DLT plugin options it includes (:50; tcpedit_opts.def, plugins/ *_opts.def) */
static const struct {
    const char *name;
    char shortopt;
    int type;
    int stacked;
} OPTS[] = {
    {"dbug", 'd', ARG_NUMBER, 0}, {"suppress-warnings", 'w', ARG_NONE, 0}, {"infile", 'i', ARG_STRING, 0},
    {"outfile", 'o', ARG_STRING, 0}, {"cachefile", 'c', ARG_STRING, 0}, {"verbose", 'v', ARG_NONE, 0},
    {"decode", 'A', ARG_STRING, 0}, {"fragroute", 0, ARG_STRING, 0}, {"fragdir", 0, ARG_STRING, 0},
    {"skip-soft-errors", 0, ARG_NONE, 0},
    /* tcpedit_opts.def */
    {"portmap", 'r', ARG_STRING, 1}, {"seed", 's', ARG_NUMBER, 0}, {"pnat", 'N', ARG_STRING, 1},
    {"srcipmap", 'S', ARG_STRING, 0}, {"dstipmap", 'D', ARG_STRING, 0}, {"endpoints", 'e', ARG_STRING, 0},
    {"tcp-sequence", 0, ARG_NUMBER, 0}, {"skipbroadcast", 'b', ARG_NONE, 0}, {"fixcsum", 'C', ARG_NONE, 0},
    {"fixhdrlen", 0, ARG_NONE, 0}, {"mtu", 'm', ARG_NUMBER, 0}, {"mtu-trunc", 0, ARG_NONE, 0},
    {"efcs", 'E', ARG_NONE, 0}, {"ttl", 0, ARG_STRING, 0}, {"tos", 0, ARG_NUMBER, 0},
    {"tclass", 0, ARG_NUMBER, 0}, {"flowlabel", 0, ARG_NUMBER, 0}, {"fixlen", 'F', ARG_STRING, 0},
    {"fuzz-seed", 0, ARG_NUMBER, 0}, {"fuzz-factor", 0, ARG_NUMBER, 0},
    /* dlt_opts.def + plugins */
    {"dlt", 0, ARG_STRING, 0}, {"skipl2broadcast", 0, ARG_NONE, 0},
    {"enet-dmac", 0, ARG_STRING, 0}, {"enet-smac", 0, ARG_STRING, 0}, {"enet-subsmac", 0, ARG_STRING, 1},
    {"enet-mac-seed", 0, ARG_NUMBER, 0}, {"enet-mac-seed-keep-bytes", 0, ARG_NUMBER, 0},
    {"enet-vlan", 0, ARG_STRING, 0}, {"enet-vlan-tag", 0, ARG_NUMBER, 0}, {"enet-vlan-cfi", 0, ARG_NUMBER, 0},
    {"enet-vlan-pri", 0, ARG_NUMBER, 0}, {"enet-vlan-proto", 0, ARG_STRING, 0},
    {"hdlc-control", 0, ARG_NUMBER, 0}, {"hdlc-address", 0, ARG_NUMBER, 0},
    {"user-dlt", 0, ARG_NUMBER, 0}, {"user-dlink", 0, ARG_STRING, 1},
};
#define NOPTS ((int)(sizeof(OPTS) / sizeof(OPTS[0])))

static tOptDesc optDesc[NOPTS];
tOptions tcprewriteOptions; /* what the generated tcprewrite_opts.c defines */

#define DESC(n) (tcprewriteOptions.pOptDesc[n])
#define HAVE_OPT_I(i) ((DESC(i).fOptState & 0xF) != 0)

static int opt_index(const char *name)
{
    for (int i = 0; i < NOPTS; i++)
        if (!strcmp(OPTS[i].name, name))
            return i;
    return -1;
}

static void usage_exit(const char *what)
{
    fprintf(stderr, "tcprewrite_abi: %s\n", what);
    exit(2);
}

/* the part of optionProcess() (libopts/autoopts.c) this program needs: the
 * descriptors end up in the state libopts leaves them in */
static int option_process(tOptions *o, int argc, char **argv)
{
    for (int i = 0; i < NOPTS; i++) {
        memset(&optDesc[i], 0, sizeof(optDesc[i]));
        *(uint16_t *)&optDesc[i].optIndex = (uint16_t)i;
        *(uint16_t *)&optDesc[i].optValue = (uint16_t)OPTS[i].shortopt;
        *(uint16_t *)&optDesc[i].optMaxCt = OPTS[i].stacked ? 0xffff : 1;
        *(const char **)&optDesc[i].pz_Name = OPTS[i].name;
        optDesc[i].fOptState = (uint32_t)OPTS[i].type << OPTST_ARG_TYPE_SHIFT;
    }
    *(int *)&o->optCt = NOPTS;
    *(tOptDesc **)&o->pOptDesc = optDesc;
    int i = 1;
    for (; i < argc; i++) {
        const char *a = argv[i], *val = NULL;
        int k = -1;
        if (a[0] == '-' && a[1] == '-') {
            const char *eq = strchr(a + 2, '=');
            char name[64];
            size_t n = eq ? (size_t)(eq - (a + 2)) : strlen(a + 2);
            if (n >= sizeof(name))
                usage_exit(a);
            memcpy(name, a + 2, n);
            name[n] = 0;
            if (!strcmp(name, "print-layout") || !strcmp(name, "check-options"))
                continue;
            k = opt_index(name);
            if (k < 0)
                usage_exit(a);
            if (OPTS[k].type != ARG_NONE)
                val = eq ? eq + 1 : (i + 1 < argc ? argv[++i] : NULL);
        } else if (a[0] == '-' && a[1] && !a[2]) {
            for (int j = 0; j < NOPTS && k < 0; j++)
                if (OPTS[j].shortopt == a[1])
                    k = j;
            if (k < 0)
                usage_exit(a);
            if (OPTS[k].type != ARG_NONE)
                val = i + 1 < argc ? argv[++i] : NULL;
        } else {
            break; /* operands */
        }
        if (OPTS[k].type != ARG_NONE && !val)
            usage_exit("missing argument");
        tOptDesc *d = &optDesc[k];
        d->fOptState |= OPTST_SET;
        d->optOccCt++;
        if (OPTS[k].type == ARG_NUMBER) {
            char *end;
            d->optArg.argInt = strtol(val, &end, 0); /* optionNumericVal: strtol(.., 0) */
            if (*end)
                usage_exit(val);
        } else if (OPTS[k].type == ARG_STRING) {
            d->optArg.argString = val;
        }
        if (OPTS[k].stacked) { /* optionStackArg: the tArgList behind optCookie */
            tArgList *al = d->optCookie;
            if (!al) {
                al = calloc(1, sizeof(tArgList) + 64 * sizeof(char *));
                al->allocCt = 6 + 64;
                d->optCookie = al;
            }
            if (al->useCt >= al->allocCt)
                usage_exit("too many stacked arguments");
            al->apzArgs[al->useCt++] = val;
            d->fOptState |= OPTST_STACKED;
        }
    }
    return i;
}

/* ---- pcap I/O (what libpcap does for the tool) ---------------------------- */
static uint32_t rd32(const uint8_t *p, int sw)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return sw ? __builtin_bswap32(v) : v;
}

static uint8_t *slurp(const char *path, size_t *n)
{
    FILE *f = fopen(path, "rb");
    if (!f)
        return NULL;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *b = malloc(sz > 0 ? (size_t)sz : 1);
    *n = fread(b, 1, (size_t)sz, f);
    fclose(f);
    return b;
}

/* src/common/cache.c:321-354 */
static tcpr_dir_t check_cache(const uint8_t *cachedata, unsigned long long packetid)
{
    const unsigned long long index = (packetid - 1) / 4;
    uint32_t bit = (uint32_t)(((packetid - 1) % 4) * 2) + 1;
    if (!(cachedata[index] & (1 << bit)))
        return TCPR_DIR_NOSEND;
    bit--;
    return (cachedata[index] & (1 << bit)) ? TCPR_DIR_C2S : TCPR_DIR_S2C;
}

#define MAXPACKET 262166 /* defines.h.in:177-182 */
#define MAX_SNAPLEN 262144

static tcpedit_t *tcpedit;

static int rewrite_packets(tcpedit_t *ctx, const uint8_t *img, size_t len, FILE *out, const uint8_t *cachedata)
{
    tcpr_dir_t cache_result = TCPR_DIR_C2S;
    struct pcap_pkthdr pkthdr, *pkthdr_ptr = &pkthdr;
    static unsigned char *pktdata_buff;
    unsigned char **pktdata;
    unsigned long long packetnum = 0;
    int rcode;
    uint32_t magic;
    memcpy(&magic, img, 4);
    const int sw = magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u;
    const int nsec = magic == 0xa1b23c4du || magic == 0x4d3cb2a1u;
    if (!pktdata_buff)
        pktdata_buff = calloc(1, MAXPACKET);
    pktdata = &pktdata_buff;
    size_t off = 24;
    while (off + 16 <= len) { /* pcap_next, then safe_pcap_next (src/common/utils.c:131-169) */
        pkthdr.ts.tv_sec = rd32(img + off, sw);
        pkthdr.ts.tv_usec = rd32(img + off + 4, sw) / (nsec ? 1000 : 1);
        pkthdr.caplen = rd32(img + off + 8, sw);
        pkthdr.len = rd32(img + off + 12, sw);
        if (pkthdr.caplen > MAX_SNAPLEN || off + 16 + pkthdr.caplen > len)
            break;
        const uint8_t *pktconst = img + off + 16;
        off += 16 + pkthdr.caplen;
        if (pkthdr.len > MAX_SNAPLEN) {
            fprintf(stderr, "safe_pcap_next ERROR: Invalid packet length: %u is greater than maximum %u\n",
                    pkthdr.len, MAX_SNAPLEN);
            fflush(out);
            exit(255);
        }
        if (!pkthdr.len || !pkthdr.caplen) {
            fprintf(stderr, "safe_pcap_next ERROR: Invalid packet length: packet length=%u capture length=%u\n",
                    pkthdr.len, pkthdr.caplen);
            fflush(out);
            exit(255);
        }
        if (pkthdr.len < pkthdr.caplen)
            pkthdr.caplen = pkthdr.len;
        packetnum++;
        memcpy(*pktdata, pktconst, pkthdr.caplen);
        if (cachedata)
            cache_result = check_cache(cachedata, packetnum);
        if (cache_result != TCPR_DIR_NOSEND) {
            if ((rcode = tcpedit_packet(ctx, &pkthdr_ptr, pktdata, cache_result)) == TCPEDIT_ERROR)
                return rcode;
            else if (rcode == TCPEDIT_SOFT_ERROR && HAVE_OPT_I(opt_index("skip-soft-errors")))
                continue;
        }
        if (pkthdr_ptr->caplen) { /* pcap_dump */
            const uint32_t rh[4] = {(uint32_t)pkthdr_ptr->ts.tv_sec, (uint32_t)pkthdr_ptr->ts.tv_usec,
                                    pkthdr_ptr->caplen, pkthdr_ptr->len};
            fwrite(rh, 1, 16, out);
            fwrite(*pktdata, 1, pkthdr_ptr->caplen, out);
        }
    }
    return 0;
}

int main(int argc, char **argv)
{
    int print_layout = 0, check_options = 0;
    for (int i = 1; i < argc; i++) {
        print_layout |= !strcmp(argv[i], "--print-layout");
        check_options |= !strcmp(argv[i], "--check-options");
    }
    if (print_layout) {
        printf("{\"sizeof_opt_desc\": %zu, \"optOccCt\": %zu, \"fOptState\": %zu, \"optArg\": %zu, "
               "\"optCookie\": %zu, \"pz_NAME\": %zu, \"pz_Name\": %zu, \"pOptDesc\": %zu, \"specOptIdx\": %zu, "
               "\"optCt\": %zu, \"apzArgs\": %zu}\n",
               sizeof(tOptDesc), offsetof(tOptDesc, optOccCt), offsetof(tOptDesc, fOptState),
               offsetof(tOptDesc, optArg), offsetof(tOptDesc, optCookie), offsetof(tOptDesc, pz_NAME),
               offsetof(tOptDesc, pz_Name), offsetof(tOptions, pOptDesc), offsetof(tOptions, specOptIdx),
               offsetof(tOptions, optCt), offsetof(tArgList, apzArgs));
        return 0;
    }

    /* tcprewrite.c:72 */
    option_process(&tcprewriteOptions, argc, argv);

    /* post_args: open the input (tcprewrite.c:244-247) and read -c (flag-code read_cache) */
    size_t in_len = 0, cache_len = 0;
    uint8_t *img = NULL, *cache = NULL;
    const uint8_t *cachedata = NULL;
    int dlt = 1;
    if (!check_options) {
        const int ki = opt_index("infile");
        if (!HAVE_OPT_I(ki))
            usage_exit("-i is required");
        img = slurp(DESC(ki).optArg.argString, &in_len);
        if (!img || in_len < 24)
            usage_exit("Unable to open input pcap file");
        uint32_t magic;
        memcpy(&magic, img, 4);
        dlt = (int)(rd32(img + 20, magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u) & 0x03ffffff);
        const int kc = opt_index("cachefile");
        if (HAVE_OPT_I(kc)) {
            cache = slurp(DESC(kc).optArg.argString, &cache_len);
            if (!cache || cache_len < 24)
                usage_exit("Unable to read cache file");
            const unsigned clen = ((unsigned)cache[22] << 8) | cache[23]; /* cache.h:63-72 */
            cachedata = cache + 24 + clen;
        }
    }

    /* tcprewrite.c:80-100 */
    if (tcpedit_init(&tcpedit, dlt) < 0) {
        fprintf(stderr, "Error initializing tcpedit: %s\n", tcpedit_geterr(tcpedit));
        tcpedit_close(&tcpedit);
        exit(255);
    }
    int rcode = tcpedit_post_args(tcpedit);
    if (rcode < 0) {
        fprintf(stderr, "Unable to parse args: %s\n", tcpedit_geterr(tcpedit));
        tcpedit_close(&tcpedit);
        exit(255);
    } else if (rcode == 1) {
        fprintf(stderr, "%s\n", tcpedit_geterr(tcpedit));
    }
    if (tcpedit_validate(tcpedit) < 0) {
        fprintf(stderr, "Unable to edit packets given options:\n%s\n", tcpedit_geterr(tcpedit));
        tcpedit_close(&tcpedit);
        exit(255);
    }
    if (check_options) { /* CPU-only check of the option bridge */
        static unsigned char cfg[1 << 16];
        const int n = tcpedit_get_dev_cfg(tcpedit, cfg, sizeof(cfg), NULL);
        const tcpedit_ref_t *ref = (const tcpedit_ref_t *)tcpedit;
        printf("seed=%u fuzz_seed=%u fuzz_factor=%u fixcsum=%d mtu=%d tos=%d validated=%d\n", ref->seed,
               ref->fuzz_seed, ref->fuzz_factor, (int)ref->fixcsum, ref->mtu, ref->tos, (int)ref->validated);
        for (int i = 0; i < n; i++)
            printf("%02x", cfg[i]);
        printf("\n");
        tcpedit_close(&tcpedit);
        return 0;
    }

    /* tcprewrite.c:103 -- the context's fields, read as the reference tool reads them */
    {
        tcpedit_ref_t *ref = (tcpedit_ref_t *)tcpedit;
        if (ref->fuzz_seed)
            fuzzing_init(ref->fuzz_seed, ref->fuzz_factor);
    }

    /* tcprewrite.c:106-147: the output file with pcap_open_dead(out_dlt, 65535)'s header */
    const int ko = opt_index("outfile");
    if (!HAVE_OPT_I(ko))
        usage_exit("-o is required");
    FILE *out = fopen(DESC(ko).optArg.argString, "wb");
    if (!out) {
        fprintf(stderr, "Unable to open output pcap file\n");
        tcpedit_close(&tcpedit);
        exit(255);
    }
    const uint32_t fh[6] = {0xa1b2c3d4u, 2 | (4u << 16), 0, 0, 65535, (uint32_t)tcpedit_get_output_dlt(tcpedit)};
    fwrite(fh, 1, 24, out);

    /* tcprewrite.c:156-161 */
    if (rewrite_packets(tcpedit, img, in_len, out, cachedata) == TCPEDIT_ERROR) {
        fprintf(stderr, "Error rewriting packets: %s\n", tcpedit_geterr(tcpedit));
        fclose(out);
        tcpedit_close(&tcpedit);
        exit(255);
    }
    fclose(out);
    tcpedit_close(&tcpedit);
    free(img);
    free(cache);
    return 0;
}
