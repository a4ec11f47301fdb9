/*
 * tcpreplay_hip.h -- tcpreplay's per-packet replay edit (--unique-ip) on an MI355X.
 *
 * The reference applies fast_edit_packet (src/send_packets.c:124-257) to every packet
 * of every pass after the first that tcpreplay makes over a capture (--loop), inline in
 * send_packets (:477-483, :758-767).  This library runs a whole pass over a
 * device-resident capture; with file output (-w, sendpacket.c:945-968) it returns the
 * bytes tcpreplay writes.  The setters mirror tcpreplay_api.h (tcpreplay_set_loop,
 * tcpreplay_set_unique_ip :649, tcpreplay_set_unique_ip_loops :657,
 * tcpreplay_set_preload_pcap) on this library's own context.
 */
#ifndef TCPREPLAY_HIP_H
#define TCPREPLAY_HIP_H
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct tcpreplay_hip_s tcpreplay_hip_t;

tcpreplay_hip_t *tcpreplay_hip_init(void);
void tcpreplay_hip_close(tcpreplay_hip_t *ctx);
const char *tcpreplay_hip_geterr(tcpreplay_hip_t *ctx);
/* the options of this path in tcpreplay's long form: --loop=N, --unique-ip,
   --unique-ip-loops=L, --preload-pcap (-K); anything else is refused */
int tcpreplay_hip_parse_args(tcpreplay_hip_t *ctx, int argc, char **argv);
int tcpreplay_hip_set_loop(tcpreplay_hip_t *ctx, uint32_t value);            /* tcpreplay_set_loop */
int tcpreplay_hip_set_unique_ip(tcpreplay_hip_t *ctx, bool value);          /* tcpreplay_set_unique_ip */
int tcpreplay_hip_set_unique_ip_loops(tcpreplay_hip_t *ctx, int value);     /* tcpreplay_set_unique_ip_loops */
int tcpreplay_hip_set_preload_pcap(tcpreplay_hip_t *ctx, bool value);       /* tcpreplay_set_preload_pcap */
/* the -w output's size bound for a capture of `len` bytes */
size_t tcpreplay_hip_output_bound(tcpreplay_hip_t *ctx, size_t len);
/* every pass over the classic pcap image (host memory) on the GPU; writes the -w file
   into out (cap bytes) and returns its length, or -1 (geterr); *failed = records whose
   unique-ip edit failed (stats->failed).  TCPREPLAY_HIP_READER_EXIT when the run ended
   where safe_pcap_next exit(-1)s (below): out then holds what tcpreplay wrote before
   exiting, tcpreplay_hip_output_len() bytes, and geterr names the record */
#define TCPREPLAY_HIP_READER_EXIT (-2)
int64_t tcpreplay_hip_replay_to_pcap(tcpreplay_hip_t *ctx, const uint8_t *pcap, size_t len, uint8_t *out, size_t cap,
                                     uint64_t *failed);
/* 1 when the last tcpreplay_hip_replay_to_pcap ended where safe_pcap_next exit(-1)s
   (send_packets.c:955,985 -> src/common/utils.c:136-156: a record with len > MAX_SNAPLEN
   or a zero len or caplen): its output is what tcpreplay wrote before exiting, and
   geterr names the record; 0 otherwise */
int tcpreplay_hip_reader_exited(tcpreplay_hip_t *ctx);
/* the -w file's length the last tcpreplay_hip_replay_to_pcap wrote (its return value on
   success; on TCPREPLAY_HIP_READER_EXIT the bytes written before the exit; 0 after -1) */
int64_t tcpreplay_hip_output_len(tcpreplay_hip_t *ctx);
#ifdef __cplusplus
}
#endif
#endif
