/*
 * san_driver.c -- host-code sanitizer runs (tests/test_sanitizers.py): the library's host
 * parsers and record walk, and the CPU oracle, built with -fsanitize=address,undefined
 * (or thread) and driven over the option lines and captures the test writes.  No HIP
 * call is made: nothing here needs a GPU.
 *
 *   san_driver <cases file> <pcap>...
 * cases file: one case a line, tab-separated fields: a tool (rewrite | prep | replay | re | ng)
 * then its arguments.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tcpedit.h"
#include "tcpprep.h"
#include "tcpreplay_hip.h"

int tcpedit_debug_index_host(tcpedit_t *t, const void *pcap, size_t len, uint64_t *n_pkts, uint64_t *n_tiles,
                             uint64_t *walk_end);
int tcpprep_regex_dfa_match(const char *re, const char *s);
int oracle_rewrite_mem(const uint8_t *in, size_t in_len, const uint8_t *cache, size_t cache_len, int argc,
                       const char **argv, uint8_t *out, size_t out_cap, size_t *out_len, int8_t *pkt_status,
                       uint64_t max_status, char *errbuf, int errlen);
long tcpprep_oracle_run(int argc, char **argv, const uint8_t *pcap, size_t len, uint8_t *out, size_t cap);
long tcpreplay_oracle_run(const uint8_t *pcap, size_t len, int loops, int unique_ip, double unique_loops,
                          int preload, uint8_t *out, size_t cap, uint64_t *failed);

static uint8_t *slurp(const char *path, size_t *len)
{
    FILE *f = fopen(path, "rb");
    if (!f)
        return NULL;
    fseek(f, 0, SEEK_END);
    *len = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *b = malloc(*len ? *len : 1);
    if (b && fread(b, 1, *len, f) != *len) {
        free(b);
        b = NULL;
    }
    fclose(f);
    return b;
}

int main(int argc, char **argv)
{
    if (argc < 3)
        return 2;
    int npcap = argc - 2;
    uint8_t **img = calloc((size_t)npcap, sizeof *img);
    size_t *len = calloc((size_t)npcap, sizeof *len);
    for (int i = 0; i < npcap; i++)
        if (!(img[i] = slurp(argv[2 + i], &len[i])))
            return 3;
    FILE *cf = fopen(argv[1], "r");
    if (!cf)
        return 4;
    char line[8192];
    long cases = 0, walked = 0;
    /* the oracle runs on the small captures only (and not at all under SAN_NO_ORACLE: the
       thread-sanitizer run is about the walker pool) */
    const int no_oracle = getenv("SAN_NO_ORACLE") != NULL;
#define ORACLE_ON(i) (!no_oracle && len[i] < ((size_t)2 << 20))
    while (fgets(line, sizeof line, cf)) {
        line[strcspn(line, "\n")] = 0;
        char *av[64];
        int ac = 0;
        for (char *tok = strtok(line, "\t"); tok && ac < 64; tok = strtok(NULL, "\t"))
            av[ac++] = tok;
        if (ac == 0)
            continue;
        cases++;
        if (!strcmp(av[0], "rewrite")) {
            tcpedit_t *t = NULL;
            if (tcpedit_init(&t, 1) == 0 && tcpedit_parse_args(t, ac - 1, av + 1, NULL) == 0 &&
                tcpedit_post_args(t) == 0 && tcpedit_validate(t) == 0) {
                for (int i = 0; i < npcap; i++) {
                    uint64_t np = 0, nt = 0, we = 0;
                    if (tcpedit_debug_index_host(t, img[i], len[i], &np, &nt, &we) == 0)
                        walked += (long)np;
                }
            }
            tcpedit_close(&t);
            for (int i = 0; i < npcap; i++) { /* the oracle on the same line */
                if (!ORACLE_ON(i))
                    continue;
                const size_t cap = 2 * len[i] + 262144 + 1024;
                uint8_t *out = malloc(cap);
                int8_t *st = malloc(len[i] / 16 + 1);
                size_t ol = 0;
                char err[512];
                oracle_rewrite_mem(img[i], len[i], NULL, 0, ac - 1, (const char **)(av + 1), out, cap, &ol, st,
                                   len[i] / 16 + 1, err, sizeof err);
                free(out);
                free(st);
            }
        } else if (!strcmp(av[0], "prep")) {
            tcpprep_hip_t *p = NULL;
            if (tcpprep_init(&p) == 0)
                tcpprep_parse_args(p, ac - 1, av + 1);
            tcpprep_close(&p);
            for (int i = 0; i < npcap; i++) {
                if (!ORACLE_ON(i))
                    continue;
                const size_t cap = 24 + 65536 + len[i] / 16 + 64;
                uint8_t *out = malloc(cap);
                tcpprep_oracle_run(ac - 1, av + 1, img[i], len[i], out, cap);
                free(out);
            }
        } else if (!strcmp(av[0], "replay")) {
            tcpreplay_hip_t *r = tcpreplay_hip_init();
            tcpreplay_hip_parse_args(r, ac - 1, av + 1);
            tcpreplay_hip_close(r);
            for (int i = 0; i < npcap; i++) {
                if (!ORACLE_ON(i))
                    continue;
                const size_t cap = 24 + 4 * len[i] + 64;
                uint8_t *out = malloc(cap);
                uint64_t failed = 0;
                tcpreplay_oracle_run(img[i], len[i], 4, 1, 2.0, ac > 1, out, cap, &failed);
                free(out);
            }
        } else if (!strcmp(av[0], "re") && ac >= 3) {
            tcpprep_regex_dfa_match(av[1], av[2]);
        } else if (!strcmp(av[0], "ng") && ac >= 2) { /* a pcapng file through the converter */
            size_t nl = 0;
            uint8_t *ng = slurp(av[1], &nl);
            void *cl = NULL;
            size_t cn = 0;
            if (ng && tcpedit_pcapng_to_pcap(ng, nl, &cl, &cn) == 0)
                walked += cn > 24;
            free(cl);
            free(ng);
        }
    }
    fclose(cf);
    for (int i = 0; i < npcap; i++)
        free(img[i]);
    free(img);
    free(len);
    printf("san_driver: %ld cases, %ld records walked\n", cases, walked);
    return 0;
}
