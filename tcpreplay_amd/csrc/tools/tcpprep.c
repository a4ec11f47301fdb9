/*
 * tcpprep -- pcap -> v04 cache file on the MI355X path.
 *
 * The caller side of the reference's tcpprep main() (src/tcpprep.c:71-200):
 * read the capture, classify every record on the GPU (tcpprep_cache_pcap,
 * include/tcpprep.h) and write the cache file.  Same options, long forms:
 * -i/--pcap, -o/--cachefile, --cidr, --mac, --port, --auto (bridge, client,
 * server, first, router), --ratio, --minmask, --maxmask, --reverse, --nonip,
 * --comment, --no-arg-comment, --include, --exclude.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tcpprep.h"

static void usage(void)
{
    fprintf(stderr, "usage: tcpprep -i <pcap> -o <cachefile> (--cidr=L | --mac=L | --port | --auto=MODE) [options]\n"
                    "  --ratio --minmask --maxmask --reverse --nonip --comment=S --no-arg-comment\n"
                    "  --include=S:|D:|B:|E:|P:<list> --exclude=...\n");
}

static void *slurp(const char *path, size_t *len)
{
    FILE *f = fopen(path, "rb");
    if (!f)
        return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    void *buf = n > 0 ? malloc((size_t)n) : NULL;
    if (!buf || fread(buf, 1, (size_t)n, f) != (size_t)n) {
        free(buf);
        fclose(f);
        return NULL;
    }
    fclose(f);
    *len = (size_t)n;
    return buf;
}

int main(int argc, char **argv)
{
    const char *in = NULL, *out = NULL;
    char **opts = calloc((size_t)argc + 1, sizeof(char *));
    int nopt = 0;
    for (int i = 1; i < argc; i++) {
        if ((!strcmp(argv[i], "-i") || !strcmp(argv[i], "--pcap")) && i + 1 < argc)
            in = argv[++i];
        else if (!strncmp(argv[i], "--pcap=", 7))
            in = argv[i] + 7;
        else if ((!strcmp(argv[i], "-o") || !strcmp(argv[i], "--cachefile")) && i + 1 < argc)
            out = argv[++i];
        else if (!strncmp(argv[i], "--cachefile=", 12))
            out = argv[i] + 12;
        else
            opts[nopt++] = argv[i];
    }
    if (!in || !out) {
        usage();
        return 1;
    }
    tcpprep_hip_t *ctx;
    if (tcpprep_init(&ctx) != 0 || tcpprep_parse_args(ctx, nopt, opts) != 0) {
        fprintf(stderr, "tcpprep: %s\n", ctx ? tcpprep_geterr(ctx) : "out of memory");
        return 1;
    }
    size_t len = 0;
    void *img = slurp(in, &len);
    if (!img) {
        fprintf(stderr, "tcpprep: cannot read %s\n", in);
        return 1;
    }
    size_t cap = tcpprep_cache_bound(ctx, len);
    void *cache = malloc(cap);
    int64_t n = cache ? tcpprep_cache_pcap(ctx, img, len, cache, cap) : -1;
    if (n < 0) {
        fprintf(stderr, "tcpprep: %s\n", tcpprep_geterr(ctx));
        return 1;
    }
    FILE *f = fopen(out, "wb");
    if (!f || fwrite(cache, 1, (size_t)n, f) != (size_t)n || fclose(f) != 0) {
        fprintf(stderr, "tcpprep: cannot write %s\n", out);
        return 1;
    }
    free(cache);
    free(img);
    free(opts);
    tcpprep_close(&ctx);
    return 0;
}
