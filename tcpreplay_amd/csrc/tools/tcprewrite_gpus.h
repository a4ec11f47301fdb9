/* tcprewrite --gpus N (tcprewrite_gpus.c): the capture image edited on devices 0..n-1 and
   written to outfile; opts are the tcpedit options (tcpedit_parse_args).  Returns the
   tool's exit status. */
#ifndef TCPREWRITE_GPUS_H
#define TCPREWRITE_GPUS_H
#include <stddef.h>
#include <stdint.h>
int tcprewrite_gpus(int n, int dlt, char **opts, int nopt, int skip_soft, const uint8_t *in, size_t in_len,
                    const uint8_t *cache, size_t cache_len, const char *outfile);
#endif
