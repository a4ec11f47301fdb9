/*
 * tcpreplay_edit_abi.c -- tcpreplay-edit's tcpedit calls and its send loop, batched,
 * against include/tcpedit.h, with file output (test program):
 *
 *   tcpreplay-edit -w <out> [--loop=N] [-K | --preload-pcap] [--include=L | --exclude=L]
 *                  [--unique-ip [--unique-ip-loops=N]] <tcpedit options> <in.pcap>
 *
 * main() follows src/tcpreplay.c:79-100 for the tcpedit calls:
 *   tcpedit_init(&tcpedit, sendpacket_get_dlt(intf1))  :81  (-w opens pcap_open_dead(
 *                                       DLT_EN10MB, MAX_SNAPLEN), sendpacket.c:945-968)
 *   tcpedit_post_args(tcpedit)          :87  (the options through tcpedit_parse_args here:
 *                                       the library's own option store)
 *   tcpedit_validate(tcpedit)           :96
 * then send_packets (send_packets.c:379-640), --loop times, with the per-packet
 * tcpedit_packet of :469-474 batched: tcpedit_replay_open holds the capture (and, with -K,
 * the preload cache that the passes after the first edit in place), tcpedit_replay_pass
 * edits one pass on the device and hands back the records as sent, which go to the -w file
 * as sendpacket's pcap_dump writes them (:485-486).  A hard error ends the run as errx()
 * does, with the records sent before it in the file.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tcpedit.h"

int main(int argc, char **argv)
{
    const char *wfile = NULL, *in = NULL;
    int loops = 1, preload = 0, nopt = 0, nrop = 0;
    char **opts = calloc((size_t)argc + 1, sizeof(char *));
    char **ropts = calloc((size_t)argc + 1, sizeof(char *)); /* tcpreplay's own per-record steps */
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-w") && i + 1 < argc)
            wfile = argv[++i];
        else if (!strncmp(argv[i], "--loop=", 7))
            loops = atoi(argv[i] + 7);
        else if (!strcmp(argv[i], "-K") || !strcmp(argv[i], "--preload-pcap"))
            preload = 1;
        else if (!strncmp(argv[i], "--include=", 10) || !strncmp(argv[i], "--exclude=", 10) ||
                 !strcmp(argv[i], "--unique-ip") || !strncmp(argv[i], "--unique-ip-loops=", 18))
            ropts[nrop++] = argv[i];
        else if (argv[i][0] == '-' && argv[i][1])
            opts[nopt++] = argv[i];
        else
            in = argv[i];
    }
    if (!wfile || !in || loops < 1) {
        fprintf(stderr, "usage: tcpreplay_edit_abi -w out [--loop=N] [-K] [tcpedit options] in.pcap\n");
        return 2;
    }
    FILE *f = fopen(in, "rb");
    if (!f)
        return 2;
    fseek(f, 0, SEEK_END);
    const size_t len = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char *img = malloc(len ? len : 1);
    if (fread(img, 1, len, f) != len)
        return 2;
    fclose(f);

    tcpedit_t *tcpedit = NULL;
    if (tcpedit_init(&tcpedit, 1 /* DLT_EN10MB */) < 0) {
        fprintf(stderr, "Error initializing tcpedit: %s\n", tcpedit_geterr(tcpedit));
        return 255;
    }
    int unused[256];
    if (tcpedit_parse_args(tcpedit, nopt, opts, unused) != 0) {
        fprintf(stderr, "Unable to parse args: %s\n", tcpedit_geterr(tcpedit));
        tcpedit_close(&tcpedit);
        return 255;
    }
    int rcode = tcpedit_post_args(tcpedit);
    if (rcode < 0) {
        fprintf(stderr, "Unable to parse args: %s\n", tcpedit_geterr(tcpedit));
        tcpedit_close(&tcpedit);
        return 255;
    }
    if (tcpedit_validate(tcpedit) < 0) {
        fprintf(stderr, "Unable to edit packets given options:\n%s\n", tcpedit_geterr(tcpedit));
        tcpedit_close(&tcpedit);
        return 255;
    }
    tcpedit_replay_t *r = tcpedit_replay_open(tcpedit, img, len, preload);
    if (!r) {
        fprintf(stderr, "Unable to open the capture: %s\n", tcpedit_geterr(tcpedit));
        tcpedit_close(&tcpedit);
        return 255;
    }
    if (tcpedit_replay_parse_args(tcpedit, r, nrop, ropts) != TCPEDIT_OK) {
        fprintf(stderr, "Unable to parse include/exclude rule: %s\n", tcpedit_geterr(tcpedit));
        tcpedit_replay_close(r);
        tcpedit_close(&tcpedit);
        return 255;
    }
    FILE *o = fopen(wfile, "wb");
    const unsigned int fh[6] = {0xa1b2c3d4u, 2 | (4u << 16), 0, 0, 262144u, 1u};
    fwrite(fh, 4, 6, o);
    const size_t cap = tcpedit_replay_bound(tcpedit, r);
    unsigned char *buf = malloc(cap ? cap : 1);
    int rc = 0;
    for (int pass = 0; pass < loops && rc == 0; pass++) {
        size_t n = 0;
        if (tcpedit_replay_pass(tcpedit, r, buf, cap, &n) != TCPEDIT_OK) {
            fprintf(stderr, "Error editing packet: %s\n", tcpedit_geterr(tcpedit));
            rc = 255;
        }
        fwrite(buf, 1, n, o);
    }
    fclose(o);
    tcpedit_replay_close(r);
    tcpedit_close(&tcpedit);
    free(buf);
    free(img);
    free(opts);
    free(ropts);
    return rc;
}
