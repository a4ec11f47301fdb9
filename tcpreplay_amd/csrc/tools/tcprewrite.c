/*
 * tcprewrite -- file -> file pcap editor on the MI355X path.
 *
 * The caller side of the reference's rewrite_packets() loop (src/tcprewrite.c:
 * 61-183 main, :260-373 rewrite_packets), driving libtcpedit_hip's batch entry
 * point instead of one tcpedit_packet() call per record: the whole capture is
 * staged in HBM and every record is edited by the gfx950 kernel in one pass.
 * Same options: -i/--infile, -o/--outfile, -c/--cachefile, --skip-soft-errors
 * and the tcpedit/en10mb option surface (tcpedit_opts.def, en10mb_opts.def).
 * Output: classic pcap, us timestamps, snaplen 65535 (tcprewrite.c:124).
 *
 * --pipeline[=MiB] reads the capture straight into page-locked memory and runs
 * the chunked H2D | edit | D2H pipeline (tcpedit_rewrite_pcap_pipelined) instead:
 * the same output bytes, without the per-record checksum warnings.
 *
 * --gpus N edits the capture on devices 0..N-1 (tcprewrite_gpus.c): byte-balanced
 * contiguous shards, one host thread and context per device, one RCCL all-reduce of the
 * counters, each shard's records copied into its range of the output file.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include "tcpedit.h"
#include "te_dev_cfg.h"
#include "tcprewrite_gpus.h"

static void usage(void)
{
    fprintf(stderr,
            "usage: tcprewrite -i <infile> -o <outfile> [-c <cachefile>] [--skip-soft-errors] [tcpedit options]\n"
            "  tcpedit options: --portmap/-r --seed/-s --pnat/-N --srcipmap/-S --dstipmap/-D --endpoints/-e\n"
            "    --tcp-sequence --skipbroadcast/-b --fixcsum/-C --fixhdrlen --mtu/-m --mtu-trunc --efcs/-E\n"
            "    --ttl --tos --tclass --flowlabel --fixlen/-F --dlt --skipl2broadcast --enet-dmac --enet-smac\n"
            "    --enet-subsmac --enet-mac-seed --enet-mac-seed-keep-bytes --enet-vlan --enet-vlan-tag\n"
            "    --enet-vlan-cfi --enet-vlan-pri --enet-vlan-proto\n"
            "  --pipeline[=MiB]: chunked H2D | edit | D2H from page-locked buffers (no per-record warnings)\n"
            "  --gpus N: edit on devices 0..N-1 (contiguous shards, one RCCL all-reduce of the counters)\n");
}

static int g_pinned; /* read into page-locked memory (--pipeline) */

static void *slurp(const char *path, size_t *len)
{
    FILE *f = fopen(path, "rb");
    if (!f)
        return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    void *buf = g_pinned ? tcpedit_host_alloc(n > 0 ? (size_t)n : 1) : malloc(n > 0 ? (size_t)n : 1);
    if (!buf || (n > 0 && fread(buf, 1, (size_t)n, f) != (size_t)n)) {
        fclose(f);
        if (g_pinned)
            tcpedit_host_free(buf);
        else
            free(buf);
        return NULL;
    }
    fclose(f);
    *len = (size_t)n;
    return buf;
}

int main(int argc, char **argv)
{
    const char *infile = NULL, *outfile = NULL, *cachefile = NULL;
    int skip_soft = 0;
    int *unused = calloc((size_t)argc + 1, sizeof(int));
    tcpedit_t *te = NULL;

    size_t pipe_mib = 0;
    int gpus = 0;
    /* the reference reads the input DLT first (pcap_datalink(pin), tcprewrite.c:80) */
    for (int i = 1; i < argc; i++) {
        if ((!strcmp(argv[i], "-i") || !strcmp(argv[i], "--infile")) && i + 1 < argc)
            infile = argv[++i];
        else if (!strncmp(argv[i], "--infile=", 9))
            infile = argv[i] + 9;
        else if (!strcmp(argv[i], "--pipeline"))
            g_pinned = 1;
        else if (!strncmp(argv[i], "--pipeline=", 11))
            g_pinned = 1, pipe_mib = strtoul(argv[i] + 11, NULL, 10);
        else if (!strcmp(argv[i], "--gpus") && i + 1 < argc)
            gpus = atoi(argv[++i]);
        else if (!strncmp(argv[i], "--gpus=", 7))
            gpus = atoi(argv[i] + 7);
    }
    if (gpus && g_pinned) {
        fprintf(stderr, "tcprewrite: --gpus and --pipeline are exclusive\n");
        return 255;
    }
    if (!infile) {
        usage();
        return 1;
    }
    size_t in_len = 0, cache_len = 0;
    uint8_t *in = slurp(infile, &in_len);
    if (!in) {
        fprintf(stderr, "Unable to open input pcap file: %s\n", infile);
        return 255;
    }
    int dlt = 1;
    if (in_len >= 24) {
        uint32_t magic, lt;
        memcpy(&magic, in, 4);
        memcpy(&lt, in + 20, 4);
        if (magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u)
            lt = __builtin_bswap32(lt);
        dlt = (int)(lt & 0x03ffffff);
    }
    if (tcpedit_init(&te, dlt) < 0) {
        fprintf(stderr, "Error initializing tcpedit: %s\n", te ? tcpedit_geterr(te) : "?");
        return 255;
    }
    int nun = tcpedit_parse_args(te, argc - 1, argv + 1, unused);
    if (nun < 0) {
        fprintf(stderr, "tcprewrite: %s\n", tcpedit_geterr(te));
        return 255;
    }
    for (int k = 0; k < nun; k++) {
        int i = unused[k] + 1;
        const char *a = argv[i];
        if (!strcmp(a, "-i") || !strcmp(a, "--infile")) {
            k++; /* value consumed above */
        } else if (!strncmp(a, "--infile=", 9)) {
        } else if ((!strcmp(a, "-o") || !strcmp(a, "--outfile")) && k + 1 < nun) {
            outfile = argv[unused[++k] + 1];
        } else if (!strncmp(a, "--outfile=", 10)) {
            outfile = a + 10;
        } else if ((!strcmp(a, "-c") || !strcmp(a, "--cachefile")) && k + 1 < nun) {
            cachefile = argv[unused[++k] + 1];
        } else if (!strncmp(a, "--cachefile=", 12)) {
            cachefile = a + 12;
        } else if (!strcmp(a, "--skip-soft-errors")) {
            skip_soft = 1;
        } else if (!strcmp(a, "--pipeline") || !strncmp(a, "--pipeline=", 11)) {
        } else if (!strcmp(a, "--gpus") && k + 1 < nun) {
            k++;
        } else if (!strncmp(a, "--gpus=", 7)) {
        } else {
            fprintf(stderr, "tcprewrite: unknown argument %s\n", a);
            usage();
            return 255;
        }
    }
    if (!outfile) {
        usage();
        return 255;
    }
    if (skip_soft && tcpedit_set_option(te, "skip-soft-errors", NULL) < 0) {
        fprintf(stderr, "tcprewrite: %s\n", tcpedit_geterr(te));
        return 255;
    }
    if (tcpedit_get_output_dlt(te) < 0 || tcpedit_post_args(te) < 0) {
        fprintf(stderr, "Unable to parse args: %s\n", tcpedit_geterr(te));
        tcpedit_close(&te);
        return 255;
    }
    tcpedit_validate(te);
    struct stat si, so;
    if (stat(outfile, &so) == 0 && stat(infile, &si) == 0 && si.st_ino == so.st_ino) {
        fprintf(stderr, "--infile and --outfile cannot be the same file\n");
        return 255;
    }
    uint8_t *cache = NULL;
    if (cachefile && !(cache = slurp(cachefile, &cache_len))) {
        fprintf(stderr, "unable to open %s\n", cachefile);
        return 255;
    }

    if (gpus > 0) { /* the tcpedit options (the arguments tcpedit_parse_args took) to every device */
        char **opts = calloc((size_t)argc, sizeof(char *));
        char *tool = calloc((size_t)argc + 1, 1);
        int nopt = 0;
        for (int k = 0; k < nun; k++)
            tool[unused[k] + 1] = 1;
        for (int i = 1; i < argc; i++)
            if (!tool[i])
                opts[nopt++] = argv[i];
        tcpedit_close(&te);
        const int grc = tcprewrite_gpus(gpus, dlt, opts, nopt, skip_soft, in, in_len, cache, cache_len, outfile);
        free(opts);
        free(tool);
        free(in);
        free(cache);
        free(unused);
        return grc;
    }
    if (g_pinned) { /* page-locked capture -> chunked pipeline -> page-locked output -> file */
        const size_t cap = tcpedit_output_bound(te, in, in_len);
        uint8_t *pout = tcpedit_host_alloc(cap > 24 ? cap : 24);
        size_t olen = 0;
        int prc = pout ? tcpedit_rewrite_pcap_pipelined(te, in, in_len, cache, cache_len, pout, cap, &olen,
                                                         pipe_mib << 20)
                       : TCPEDIT_ERROR;
        FILE *f = fopen(outfile, "wb");
        if (!f || fwrite(pout, 1, olen, f) != olen) {
            fprintf(stderr, "Unable to write output pcap file: %s\n", outfile);
            return 255;
        }
        fclose(f);
        if (prc != 0)
            fprintf(stderr, "Error rewriting packets: %s\n", tcpedit_geterr(te));
        tcpedit_host_free(pout);
        tcpedit_host_free(in);
        tcpedit_host_free(cache);
        tcpedit_close(&te);
        free(unused);
        return prc != 0 ? 255 : 0;
    }
    tcpedit_batch_t *b = tcpedit_batch_open(te, in, in_len, cache, cache_len, 0);
    if (!b) {
        fprintf(stderr, "tcprewrite: %s\n", tcpedit_geterr(te));
        return 255;
    }
    int rc = tcpedit_batch_run(te, b);
    tcpedit_batch_result_t r;
    tcpedit_batch_result(b, &r);
    if (r.unsupported) {
        fprintf(stderr, "Error rewriting packets: %s\n", tcpedit_geterr(te));
        return 255;
    }
    /* per-record warnings, in record order (tcpedit.c:351-353) */
    const uint8_t *st = tcpedit_batch_status(b);
    uint64_t last = r.first_error >= 0 ? (uint64_t)r.first_error : r.packets;
    for (uint64_t i = 0; st && i < last; i++)
        if (st[i] & TE_ST_WARNED)
            fprintf(stderr, "Warning: packet %llu: checksums left unchanged (caplen/IP length mismatch, "
                            "fragment or short L4). Consider option '--fixhdrlen'.\n",
                    (unsigned long long)(i + 1));
    uint8_t *out = malloc(r.out_len ? r.out_len : 1);
    size_t n = tcpedit_batch_output(b, out, r.out_len);
    FILE *f = fopen(outfile, "wb");
    if (!f || fwrite(out, 1, n, f) != n) {
        fprintf(stderr, "Unable to write output pcap file: %s\n", outfile);
        return 255;
    }
    fclose(f);
    tcpedit_batch_close(b);
    if (rc != 0) {
        fprintf(stderr, "Error rewriting packets: %s\n", tcpedit_geterr(te));
        tcpedit_close(&te);
        return 255;
    }
    tcpedit_close(&te);
    free(out);
    free(in);
    free(cache);
    free(unused);
    return 0;
}
