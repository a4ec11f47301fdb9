/*
 * tcprewrite_gpus.c -- `tcprewrite --gpus N`: one process edits a capture on N GPUs.
 *
 * The multi-GPU rewrite of SURVEY.md section 8(e) for a C host (no Python, no
 * torch.distributed): one host thread and one tcpedit context per device, the capture
 * cut into N contiguous byte-balanced runs of whole records (tcpedit_pcap_shards), each
 * run staged on its device in place (tcpedit_batch_open_segment) and edited start to
 * finish there.  The records are independent for every edit in scope; the two edits
 * that carry state across records take a host-side prefix before the edit (--fuzz-seed's
 * single RNG stream, fuzzing.c:8-20,87; the en10mb dst_modified carry, en10mb.c:612-615,
 * SURVEY Q18), exactly as dist.py's one pre-edit exchange.  The job's counters are summed
 * by one RCCL all-reduce over the devices (ncclCommInitAll: xGMI between the GPUs of the
 * node), and every thread copies its output records straight into its range of an mmap of
 * the output file (tcpedit_batch_output_records), placed by tcpedit_shard_place with
 * tcprewrite's hard-error rule (tcprewrite.c:156-160).
 */
#define _GNU_SOURCE
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "tcpedit.h"
#include "te_dev_cfg.h"
#include "tcprewrite_gpus.h"

#define NCNT 9 /* packets .. unsupported, tcpedit_batch_result_t's counters */

typedef struct {
    int k;
    struct job_s *job;
    tcpedit_t *te;
    tcpedit_batch_t *b;
    int opened, rc;
    int jfail;          /* the Juniper state seeding failed (read by all after the inner barrier) */
    int ffail, skipped; /* the fuzz skip (and the carry-out after it) failed / was applied */
    int64_t reach;
    int carry;
    int jnpr;                                 /* DLT_JUNIPER_ETHER: the decoder-state exchange runs */
    int jvalid;                               /* this shard has a whole inner decode ... */
    uint8_t jstate[TCPEDIT_JNPR_STATE_BYTES]; /* ... and the state its last one leaves */
    tcpedit_batch_result_t r;
    uint64_t seg;
    const uint8_t *status;
    uint64_t *d_cnt;    /* the counter all-reduce's device buffer and stream, set up before */
    hipStream_t cst;    /* the first barrier: a shard without them takes no device into it */
    char err[512];
} shard_t;

typedef struct job_s {
    int n, dlt, skip_soft, nopt;
    char **opts;
    const uint8_t *in;
    size_t in_len;
    const uint8_t *cache;
    size_t cache_len;
    uint64_t *off, *base;
    int64_t total;
    ncclComm_t *comms;
    pthread_barrier_t bar;
    shard_t *sh;
    /* placement (thread 0, between barriers) */
    uint64_t *place_off, *place_write, file_end;
    uint8_t *omap;
    int ofd;
    const char *outfile;
    int place_ok;
    uint64_t job_cnt[NCNT];
} job_t;

static void *shard_main(void *arg)
{
    shard_t *S = arg;
    job_t *J = S->job;
    const int k = S->k;
    int unused_n = 0;
    /* ---- context and batch on device k ---- */
    if (tcpedit_set_device(k) < 0) {
        snprintf(S->err, sizeof S->err, "device %d: hipSetDevice failed", k);
    } else if (tcpedit_init(&S->te, J->dlt) < 0) {
        snprintf(S->err, sizeof S->err, "device %d: %s", k, S->te ? tcpedit_geterr(S->te) : "tcpedit_init failed");
    } else {
        int *unused = calloc((size_t)J->nopt + 1, sizeof(int));
        unused_n = tcpedit_parse_args(S->te, J->nopt, J->opts, unused);
        free(unused);
        if (unused_n != 0 || (J->skip_soft && tcpedit_set_option(S->te, "skip-soft-errors", NULL) < 0) ||
            tcpedit_post_args(S->te) < 0) {
            snprintf(S->err, sizeof S->err, "device %d: %s", k, tcpedit_geterr(S->te));
        } else {
            tcpedit_validate(S->te);
            S->b = tcpedit_batch_open_segment(S->te, J->in, J->in + J->off[k], J->off[k + 1] - J->off[k], J->cache,
                                              J->cache_len, J->base[k]);
            if (!S->b)
                snprintf(S->err, sizeof S->err, "device %d: %s", k, tcpedit_geterr(S->te));
            else if (k > 0) /* the earlier shards: read only by a stale-buffer replay */
                tcpedit_batch_set_prefix(S->te, S->b, J->in + 24, J->off[k] - 24);
        }
    }
    if (S->b) {
        S->reach = tcpedit_batch_fuzz_reach(S->te, S->b);
        /* DLT_JUNIPER_ETHER: the shards' decoder states go round first (below); the
           dst_modified carry-out reads the seeded state, so it waits for it */
        S->jnpr = J->dlt == 178;
        S->jvalid = S->jnpr ? tcpedit_batch_jnpr_out(S->te, S->b, S->jstate, sizeof S->jstate) : 0;
        S->carry = S->jnpr ? 2 : tcpedit_batch_l2carry_out(S->te, S->b);
        S->opened = S->reach >= 0 && S->carry >= 0 && S->jvalid >= 0;
        if (!S->opened)
            snprintf(S->err, sizeof S->err, "device %d: %s", k, tcpedit_geterr(S->te));
    }
    if (S->opened) { /* the all-reduce's device buffer and stream (RCCL reads device memory only) */
        const char *inj = getenv("TCPREWRITE_GPUS_FAIL_COUNTERS"); /* (tests: this shard's setup fails) */
        const int fail = inj && *inj && atoi(inj) == k;
        if (fail || hipSetDevice(k) != hipSuccess ||
            hipStreamCreateWithFlags(&S->cst, hipStreamNonBlocking) != hipSuccess ||
            hipMalloc((void **)&S->d_cnt, NCNT * sizeof(uint64_t)) != hipSuccess) {
            snprintf(S->err, sizeof S->err, "device %d: no device buffer for the counter all-reduce", k);
            S->opened = 0;
        }
    }
    /* ---- the pre-edit prefix: earlier shards' fuzz draws and dst_modified carry ---- */
    pthread_barrier_wait(&J->bar);
    int all_open = 1;
    uint64_t skip = 0;
    int carry_in = 0;
    for (int j = 0; j < J->n; j++)
        all_open &= J->sh[j].opened;
    if (all_open && J->dlt == 178) {
        /* the nearest earlier shard's Juniper decoder state, then this shard's carry-out.
           A failure here goes to jfail, not opened: the other threads may still be reading
           every shard's opened flag above, and all of them fold jfail in only
           after the barrier, so they agree on all_open and on joining the all-reduce */
        const uint8_t *src = NULL;
        for (int j = k - 1; j >= 0 && !src; j--)
            if (J->sh[j].jvalid == 1)
                src = J->sh[j].jstate;
        const char *inj = getenv("TCPREWRITE_GPUS_FAIL_JNPR"); /* (tests: this shard's seeding fails) */
        if ((inj && *inj && atoi(inj) == k) || tcpedit_set_jnpr_state(S->te, src, TCPEDIT_JNPR_STATE_BYTES, 0) < 0 ||
            (S->carry = tcpedit_batch_l2carry_out(S->te, S->b)) < 0) {
            snprintf(S->err, sizeof S->err, "device %d: %s", k,
                     inj && *inj && atoi(inj) == k ? "Juniper state seeding failed (injected)" : tcpedit_geterr(S->te));
            S->jfail = 1;
        }
        pthread_barrier_wait(&J->bar);
        for (int j = 0; j < J->n; j++)
            all_open &= !J->sh[j].jfail;
        if (S->jfail)
            S->opened = 0; /* (no thread reads opened again before the placement barrier) */
    }
    for (int j = 0; j < k; j++)
        skip += (uint64_t)J->sh[j].reach;
    int any_fz = 0;
    for (int j = 0; j < J->n; j++)
        any_fz |= J->sh[j].reach > 0;
    if (all_open && any_fz) {
        /* --fuzz-seed: this shard's RNG stream starts after the earlier shards' draws; with the
           dst_modified carry a fuzzed record's second encode writes it, so a
           shard that fuzzes after earlier draws finds its carry-out again from there */
        if ((skip && tcpedit_fuzz_skip(S->te, skip) < 0) ||
            (S->reach > 0 && skip && (S->carry = tcpedit_batch_l2carry_out(S->te, S->b)) < 0)) {
            snprintf(S->err, sizeof S->err, "device %d: %s", k, tcpedit_geterr(S->te));
            S->ffail = 1;
        }
        S->skipped = 1;
        pthread_barrier_wait(&J->bar);
        for (int j = 0; j < J->n; j++)
            all_open &= !J->sh[j].ffail;
        if (S->ffail)
            S->opened = 0;
    }
    for (int j = k - 1; j >= 0; j--)
        if (J->sh[j].carry == 0 || J->sh[j].carry == 1) {
            carry_in = J->sh[j].carry;
            break;
        }
    S->rc = TCPEDIT_ERROR;
    uint64_t cnt[NCNT] = {0};
    if (all_open) {
        if ((skip && !S->skipped && tcpedit_fuzz_skip(S->te, skip) < 0) || tcpedit_set_l2carry(S->te, carry_in) < 0) {
            snprintf(S->err, sizeof S->err, "device %d: %s", k, tcpedit_geterr(S->te));
        } else {
            S->rc = tcpedit_batch_run(S->te, S->b);
            tcpedit_batch_result(S->b, &S->r);
            if (S->rc != 0)
                snprintf(S->err, sizeof S->err, "%s", tcpedit_geterr(S->te));
            S->seg = S->r.out_len > 24 ? S->r.out_len - 24 : 0;
            S->status = tcpedit_batch_status(S->b);
            const uint64_t v[NCNT] = {S->r.packets,  S->r.bytes_in,    S->r.bytes_out,
                                      S->r.written,  S->r.edited,      S->r.soft_errors,
                                      S->r.warnings, S->r.errors,      S->r.unsupported};
            memcpy(cnt, v, sizeof cnt);
        }
    }
    /* ---- the job's counters: one RCCL all-reduce over the devices.  Every shard opened
       (and has its device buffer) or none takes part: each thread decided all_open from the
       same flags after the barrier, so no device is left waiting in the collective, and a
       failed shard ends the job with its message instead of a fault ---- */
    if (all_open) {
        int ok = hipSetDevice(k) == hipSuccess &&
                 hipMemcpyAsync(S->d_cnt, cnt, sizeof cnt, hipMemcpyHostToDevice, S->cst) == hipSuccess;
        ncclResult_t nr = ncclAllReduce(S->d_cnt, S->d_cnt, NCNT, ncclUint64, ncclSum, J->comms[k], S->cst);
        ok = ok && nr == ncclSuccess && hipMemcpyAsync(cnt, S->d_cnt, sizeof cnt, hipMemcpyDeviceToHost, S->cst) ==
                                            hipSuccess &&
             hipStreamSynchronize(S->cst) == hipSuccess;
        if (!ok && !S->err[0])
            snprintf(S->err, sizeof S->err, "device %d: counter all-reduce failed (%s)", k, ncclGetErrorString(nr));
        if (!ok)
            S->rc = TCPEDIT_ERROR, S->opened = 0;
        if (k == 0)
            memcpy(J->job_cnt, cnt, sizeof cnt);
    }
    hipFree(S->d_cnt);
    S->d_cnt = NULL;
    if (S->cst)
        hipStreamDestroy(S->cst);
    S->cst = NULL;
    /* ---- placement and the output file (thread 0), then every shard's D2H into it ---- */
    pthread_barrier_wait(&J->bar);
    if (k == 0) {
        J->place_ok = 1;
        uint64_t *seg = calloc((size_t)J->n, sizeof(uint64_t));
        int *err = calloc((size_t)J->n, sizeof(int));
        for (int j = 0; j < J->n; j++) {
            J->place_ok &= J->sh[j].opened && (J->sh[j].rc == 0 || J->sh[j].r.first_error >= 0);
            seg[j] = J->sh[j].seg;
            err[j] = J->sh[j].rc != 0;
        }
        J->file_end = tcpedit_shard_place(J->n, seg, err, J->place_off, J->place_write);
        free(seg);
        free(err);
        uint8_t hdr[24];
        J->ofd = -1;
        J->omap = NULL;
        if (J->place_ok && tcpedit_batch_output(S->b, hdr, 24) == 24) {
            J->ofd = open(J->outfile, O_RDWR | O_CREAT | O_TRUNC, 0644);
            if (J->ofd >= 0 && ftruncate(J->ofd, (off_t)J->file_end) == 0 && pwrite(J->ofd, hdr, 24, 0) == 24) {
                J->omap = mmap(NULL, J->file_end, PROT_READ | PROT_WRITE, MAP_SHARED, J->ofd, 0);
                if (J->omap == MAP_FAILED)
                    J->omap = NULL;
            }
        }
        if (!J->omap)
            J->place_ok = 0;
    }
    pthread_barrier_wait(&J->bar);
    if (J->place_ok && J->place_write[k]) {
        const size_t got = tcpedit_batch_output_records(S->b, J->omap + J->place_off[k], J->place_write[k]);
        if (got != J->place_write[k]) {
            snprintf(S->err, sizeof S->err, "device %d: wrote %zu of %llu output bytes", k, got,
                     (unsigned long long)J->place_write[k]);
            S->opened = 0;
        }
    }
    return NULL;
}

int tcprewrite_gpus(int n, int dlt, char **opts, int nopt, int skip_soft, const uint8_t *in, size_t in_len,
                    const uint8_t *cache, size_t cache_len, const char *outfile)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < n) {
        fprintf(stderr, "tcprewrite: --gpus %d: %d HIP device(s) visible\n", n, ndev);
        return 255;
    }
    job_t J;
    memset(&J, 0, sizeof J);
    J.n = n;
    J.dlt = dlt;
    J.opts = opts;
    J.nopt = nopt;
    J.skip_soft = skip_soft;
    J.in = in;
    J.in_len = in_len;
    J.cache = cache;
    J.cache_len = cache_len;
    J.outfile = outfile;
    J.off = calloc((size_t)n + 1, sizeof(uint64_t));
    J.base = calloc((size_t)n, sizeof(uint64_t));
    J.place_off = calloc((size_t)n, sizeof(uint64_t));
    J.place_write = calloc((size_t)n, sizeof(uint64_t));
    J.sh = calloc((size_t)n, sizeof(shard_t));
    J.comms = calloc((size_t)n, sizeof(ncclComm_t));
    int *devs = calloc((size_t)n, sizeof(int));
    J.total = tcpedit_pcap_shards(in, in_len, n, J.off, J.base);
    if (J.total < 0) {
        fprintf(stderr, "tcprewrite: not a pcap file\n");
        return 255;
    }
    for (int k = 0; k < n; k++)
        devs[k] = k;
    ncclResult_t nr = ncclCommInitAll(J.comms, n, devs);
    if (nr != ncclSuccess) {
        fprintf(stderr, "tcprewrite: ncclCommInitAll(%d): %s\n", n, ncclGetErrorString(nr));
        return 255;
    }
    pthread_barrier_init(&J.bar, NULL, (unsigned)n);
    pthread_t *th = calloc((size_t)n, sizeof(pthread_t));
    for (int k = 0; k < n; k++) {
        J.sh[k].k = k;
        J.sh[k].job = &J;
        pthread_create(&th[k], NULL, shard_main, &J.sh[k]);
    }
    for (int k = 0; k < n; k++)
        pthread_join(th[k], NULL);
    int rc = 0;
    const char *why = NULL;
    for (int k = 0; k < n && !why; k++)
        if (!J.sh[k].opened)
            why = J.sh[k].err[0] ? J.sh[k].err : "a shard failed";
    if (why) {
        fprintf(stderr, "tcprewrite: %s\n", why);
        rc = 255;
    } else if (J.job_cnt[8]) {
        fprintf(stderr, "Error rewriting packets: a record's stale static-buffer read is not reproducible across a "
                        "shard cut\n");
        rc = 255;
    } else {
        /* per-record warnings in record order (tcpedit.c:351-353), then the first hard error */
        for (int k = 0; k < n; k++) {
            const shard_t *S = &J.sh[k];
            const uint64_t last = S->r.first_error >= 0 ? (uint64_t)S->r.first_error : S->r.packets;
            for (uint64_t i = 0; S->status && i < last; i++)
                if (S->status[i] & TE_ST_WARNED)
                    fprintf(stderr,
                            "Warning: packet %llu: checksums left unchanged (caplen/IP length mismatch, fragment or "
                            "short L4). Consider option '--fixhdrlen'.\n",
                            (unsigned long long)(J.base[k] + i + 1));
            if (S->rc != 0) {
                fprintf(stderr, "Error rewriting packets: %s\n", S->err);
                rc = 255;
                break;
            }
        }
        if (!J.place_ok && !rc) {
            fprintf(stderr, "Unable to write output pcap file: %s\n", outfile);
            rc = 255;
        }
    }
    if (J.omap) {
        msync(J.omap, J.file_end, MS_SYNC);
        munmap(J.omap, J.file_end);
    }
    if (J.ofd >= 0)
        close(J.ofd);
    for (int k = 0; k < n; k++) { /* (each shard's objects freed with its device current) */
        hipSetDevice(k);
        if (J.sh[k].b)
            tcpedit_batch_close(J.sh[k].b);
        if (J.sh[k].te)
            tcpedit_close(&J.sh[k].te);
        ncclCommDestroy(J.comms[k]);
    }
    pthread_barrier_destroy(&J.bar);
    free(th);
    free(devs);
    free(J.comms);
    free(J.sh);
    free(J.place_write);
    free(J.place_off);
    free(J.base);
    free(J.off);
    return rc;
}
