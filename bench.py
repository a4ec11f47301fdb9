"""bench.py -- device-resident tcpedit rewrite throughput on MI355X.

Metric (BASELINE.json): Mpackets/s of the device-resident tcpedit rewrite
(+ fixcsum), with the GB/s roofline of the kernel.  At N=1 the workload is
BASELINE configs[1]: `--seed=42 --fixcsum` over 1M x 64 B synthetic UDP
records.  A "step" is one pass of the whole device pipeline (one kernel:
parse + edit + checksum + scan + compaction) over that batch, inputs already
resident in HBM.  With --gpus N (one process per GPU, torch.distributed over
RCCL) every rank rewrites its own shard of the N = 1 workload (1M x 64 B: weak
scaling, like with like) -- packets are independent, so
there is no data-path collective, only one all-reduce of the counters per job
-- and `value` is the aggregate packets/s over the max-over-ranks time; a
`strong_c4` side line runs BASELINE configs[3] (100M records split over the
ranks).

Every workload's first (untimed) run is checked byte for byte against the
oracle (tests/oracle_lib.check_rewrite) before it is timed: `verified` and
`verified_records` in the JSON line (--no-verify skips it).

Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes
import json
import os
import struct
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)

WORKLOADS = {
    # name: (generator, kwargs, tcpedit args, description)
    "c2": ("pcap_fixed", dict(size=64), ["--seed=42", "--fixcsum"],
           "--seed=42 --fixcsum on 1M x 64B synthetic UDP pcap (BASELINE configs[1])"),
    "c3": ("pcap_imix", dict(), ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353,80:8080", "--fixcsum"],
           "--pnat + --portmap + --fixcsum on IMIX 64/570/1514 7:4:1 (BASELINE configs[2])"),
    "c5": ("pcap_mixed_v4v6", dict(size=1514), ["--fixcsum"],
           "--fixcsum on 1514B mixed IPv4/IPv6 TCP/UDP (BASELINE configs[4])"),
    "c4": ("pcap_imix", dict(), ["--endpoints=10.10.0.1:10.10.0.2", "--enet-dmac=00:12:13:14:15:16,00:22:33:44:55:66",
                                 "--enet-smac=00:22:33:44:55:66,00:12:13:14:15:16", "--enet-vlan=add",
                                 "--enet-vlan-tag=45", "--enet-vlan-pri=5", "--enet-vlan-cfi=1", "--fixcsum"],
           "tcpreplay-edit chain (endpoints + tcpprep cache, enet MACs, VLAN add, fixcsum) on IMIX: one GPU's "
           "12.5M-record share of the 100M-record 8-GPU job (BASELINE configs[3])"),
    "c2x10": ("pcap_fixed", dict(size=64), ["--seed=42", "--fixcsum"],
              "--seed=42 --fixcsum on 10M x 64B (C2 at 1.6 GB moved: launch amortised, HBM- not cache-resident; "
              "SURVEY 8(d))"),
    "fz": ("pcap_imix", dict(), ["--fuzz-seed=42", "--fuzz-factor=2"],
           "--fuzz-seed=42 --fuzz-factor=2 (the l7fuzzing golden's options) on IMIX 64/570/1514 7:4:1: reach pass, "
           "RNG-state scan, edit pass (SURVEY 8(f) rank 4)"),
    # common tcprewrite lines without --fixcsum or with size changes
    "seed": ("pcap_fixed", dict(size=64), ["--seed=42"],
             "--seed=42 without --fixcsum (incremental checksums, SURVEY Q13) on 1M x 64B"),
    "hdr": ("pcap_imix", dict(), ["--ttl=+1", "--tos=7"],
            "--ttl=+1 --tos=7 on IMIX 64/570/1514 7:4:1 (TTL change -> full recompute, tcpedit.c:195,338)"),
    "vdel": ("pcap_imix", dict(vlan=0xB02D), ["--enet-vlan=del", "--fixcsum"],
             "--enet-vlan=del --fixcsum on 802.1Q-tagged IMIX 68/574/1518 (every record -4 bytes)"),
    "efcs": ("pcap_imix", dict(fcs=True), ["--efcs", "--fixcsum"],
             "--efcs --fixcsum on IMIX 68/574/1518 7:4:1 frames captured with their FCS (every record -4 bytes)"),
    "macseed": ("pcap_imix", dict(), ["--enet-mac-seed=42", "--fixcsum"],
                "--enet-mac-seed=42 --fixcsum on IMIX 64/570/1514 7:4:1 (MAC seed masks, en10mb.c:674-689)"),
    # a size change that differs by record: the wave lane's SZ_MTU instances, tiles placed by the
    # device-predicted cuts (te_mtu_cuts; TCPEDIT_HIP_NO_MTU_FAST=1: the generic lane's scan + look-back)
    "mtu": ("pcap_imix", dict(), ["--mtu=1000", "--mtu-trunc", "--fixcsum"],
            "--mtu=1000 --mtu-trunc --fixcsum on IMIX 64/570/1514 7:4:1 (1514 B records cut to 1014 B: "
            "per-record sizes; wave lane, tiles at the predicted cuts' prefix)"),
}
# every rank's share at N > 1: the N = 1 workload itself (BASELINE configs[1]'s 1M x 64 B
# for c2), so the driver's 1/2/4/8 curve weak-scales like with like; the
# HBM-resident 10M-record form is the c2x10 side line (--packets 10000000 at any N)
PER_RANK_PACKETS = {}
DEFAULT_PACKETS = {"c2": 1_000_000, "c3": 10_000_000, "c5": 1_000_000, "c4": 12_500_000, "c2x10": 10_000_000,
                   "fz": 10_000_000, "seed": 1_000_000, "hdr": 4_000_000, "vdel": 4_000_000, "efcs": 4_000_000, "macseed": 4_000_000,
                   "mtu": 4_000_000}
CACHED = {"c4"}  # workloads with a tcpprep cache (synth.tcpprep_cache: C2S/S2C runs by flow)


def make_pcap(workload, n, seed):
    from tcpreplay_amd import synth
    gen, kw, _, _ = WORKLOADS[workload]
    return getattr(synth, gen)(n, seed=seed, **kw)


STRONG_BLOCK = 1_250_000  # records generated once per rank and repeated (--strong)
STRONG_VERIFY_MAX = 25_000_000  # --strong / the strong side line: shares checked against the oracle


def make_share(workload, total, rank, world, seed):
    """--strong: rank's share [rank*total/world, (rank+1)*total/world) of one `total`-record
    capture, generated on this rank alone so no host holds more than its share: a
    STRONG_BLOCK-record block of the workload repeated (the record mix and sizes of the
    config; the endpoints/cache edits vary by global record number through the cache),
    returned as (file header, records, first global record, records)."""
    first, last = total * rank // world, total * (rank + 1) // world
    cnt = last - first
    blk = min(cnt, STRONG_BLOCK) if cnt else 0
    block = make_pcap(workload, max(blk, 1), seed + rank)
    body = block[24:] if blk else b""
    reps, tail = (cnt // blk, cnt % blk) if blk else (0, 0)
    parts = [body] * reps
    if tail:  # the first `tail` records of the block
        off, k = 24, 0
        while k < tail:
            off += 16 + int.from_bytes(block[off + 8:off + 12], "little")
            k += 1
        parts.append(block[24:off])
    return block[:24], b"".join(parts), first, cnt


def verify_threads():
    """checker threads: the CPUs this process may run on, at most 16 (the GPU box's CPU share)"""
    return max(1, min(16, len(os.sched_getaffinity(0))))


def check_output(b, pcap, args, cache, pkt_base=0, hdr=None):
    """Parity on the bench's own clock (outside the timed region): the device output of the
    batch's first run against the oracle (tests/oracle_lib.check_rewrite, the CPU restatement
    of tcpedit_packet) on the same input and options, byte for byte.  Records are
    independent unless --fuzz-seed or a stale static-buffer read (Q8) carries state, so the
    oracle runs on byte-balanced shards of whole records on `verify_threads()` threads,
    else on one.  Returns the records checked; raises on any difference."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    r = b.result()
    dev = b.output_np()
    if hdr is not None:  # a --strong share: file header + this rank's records
        import numpy as np
        src = np.empty(24 + len(pcap), np.uint8)
        src[:24] = np.frombuffer(hdr, np.uint8)[:24]
        src[24:] = np.frombuffer(pcap, np.uint8)
        pcap = src
    sharded = not any(a.startswith("--fuzz-seed") for a in args) and r.stale_records == 0
    n = oracle_lib.check_rewrite(pcap, args, cache, dev, threads=verify_threads(), sharded=sharded,
                                 pkt_base=pkt_base)
    if n != r.packets:
        raise RuntimeError(f"checker walked {n} records, the device {r.packets}")
    return n


def check_output_bytes(pcap, args, cache, out):
    """check_output for an output image already on the host"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    return oracle_lib.check_rewrite(pcap, args, cache, out, threads=verify_threads())


def run_workload(workload, n, steps, warmup, seed, device, verify=True, share=None, total=None):
    """Open the workload's batch, run it once (untimed) and, with `verify`, check that run's
    output against the oracle.  Returns (context, batch, result, pcap, records verified)."""
    import tcpreplay_amd as TA
    from tcpreplay_amd import synth
    args = WORKLOADS[workload][2]
    if share is not None:  # --strong: this rank's records of the one capture, in place
        hdr, body, first, n = share
        cache = synth.tcpprep_cache(total, seed=seed) if workload in CACHED else None
        te = TA.TcpEdit(args, device=device)
        b = TA.Batch(te, body, cache, pkt_base=first, hdr=hdr)
        pcap = None
    else:
        pcap = make_pcap(workload, n, seed)
        cache = synth.tcpprep_cache(n, seed=seed) if workload in CACHED else None
        te = TA.TcpEdit(args, device=device)
        b = TA.Batch(te, pcap, cache)
    rc = b.run()  # first (untimed) run: also the run the checker compares
    r = b.result()
    if rc != 0 or r.unsupported or r.errors:
        raise RuntimeError(f"{workload}: device run failed rc={rc} ({te.geterr()})")
    checked = 0
    if verify:
        if share is not None:
            checked = check_output(b, share[1], args, cache, pkt_base=share[2], hdr=share[0])
        else:
            checked = check_output(b, pcap, args, cache)
    if warmup:
        b.time(warmup)
    return te, b, r, pcap, checked


def _pcap_shards(pcap, parts):
    """Split a pcap image into `parts` pcaps of contiguous whole records (byte-balanced)."""
    swapped = pcap[:4] in (b"\xa1\xb2\xc3\xd4", b"\xa1\xb2\x3c\x4d")  # big-endian file
    fmt = ">I" if swapped else "<I"
    hdr, pos, n = pcap[:24], 24, len(pcap)
    target = (n - 24) / parts
    cuts, nxt = [24], 24 + target
    while pos + 16 <= n:
        if pos >= nxt and len(cuts) < parts:
            cuts.append(pos)
            nxt += target
        pos += 16 + struct.unpack_from(fmt, pcap, pos + 8)[0]
    cuts.append(n)
    return [hdr + pcap[a:b] for a, b in zip(cuts, cuts[1:]) if b > a]


def copy_floor(src_addr, n_in, dst_addr, n_out, reps=5):
    """The box's PCIe floor for the end-to-end path: the capture up and its output down, one
    hipMemcpyAsync each on two streams at once, from and to the same page-locked buffers the
    pipelined run uses (median ms).  No edit can beat it; end_to_end.ms is read against it."""
    hip = ctypes.CDLL("libamdhip64.so")
    din, dout, s1, s2 = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    if hip.hipMalloc(ctypes.byref(din), ctypes.c_size_t(n_in)) or hip.hipMalloc(ctypes.byref(dout),
                                                                                 ctypes.c_size_t(n_out)):
        return None
    hip.hipStreamCreateWithFlags(ctypes.byref(s1), 1)
    hip.hipStreamCreateWithFlags(ctypes.byref(s2), 1)
    ts = []
    for _ in range(reps + 1):
        hip.hipDeviceSynchronize()
        t0 = time.perf_counter()
        hip.hipMemcpyAsync(din, ctypes.c_void_p(src_addr), ctypes.c_size_t(n_in), 1, s1)
        hip.hipMemcpyAsync(ctypes.c_void_p(dst_addr), dout, ctypes.c_size_t(n_out), 2, s2)
        hip.hipDeviceSynchronize()
        ts.append(time.perf_counter() - t0)
    hip.hipStreamDestroy(s1)
    hip.hipStreamDestroy(s2)
    hip.hipFree(din)
    hip.hipFree(dout)
    return sorted(ts[1:])[reps // 2] * 1e3


def cpu_baseline(pcap, args, n_pkts, budget_s=10.0, threads=1):
    """The oracle (C restatement of tcpedit_packet) on the same workload: only the C call
    is timed, over preallocated buffers; with threads > 1 each thread rewrites its own
    byte-balanced shard of whole records (ctypes drops the GIL during the call)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes
    import oracle_lib
    from concurrent.futures import ThreadPoolExecutor
    lib = oracle_lib.load()
    argv = (ctypes.c_char_p * max(1, len(args)))(*[a.encode() for a in args])
    shards = _pcap_shards(pcap, threads) if threads > 1 else [pcap]
    jobs = []
    for sh in shards:
        cap = len(sh) * 2 + 262144
        npk = max(1, len(sh) // 16)
        jobs.append((ctypes.create_string_buffer(sh, len(sh)), len(sh), ctypes.create_string_buffer(cap), cap,
                     (ctypes.c_int8 * npk)(), npk, ctypes.create_string_buffer(1024)))

    def one(j):
        inbuf, inlen, out, cap, status, npk, err = j
        olen = ctypes.c_size_t(0)
        rc = lib.oracle_rewrite_mem(inbuf, inlen, None, 0, len(args), argv, out, cap, ctypes.byref(olen),
                                    status, npk, err, 1024)
        if rc < 0:
            raise RuntimeError("oracle failed: " + err.value.decode(errors="replace"))

    with ThreadPoolExecutor(max_workers=len(jobs)) as ex:
        list(ex.map(one, jobs))  # warm (page-in)
        runs, t0 = 0, time.perf_counter()
        while True:
            list(ex.map(one, jobs))
            runs += 1
            el = time.perf_counter() - t0
            if el >= budget_s:
                break
    return runs * n_pkts / el / 1e6, runs, el, len(jobs)


def strong_side(opt, world, rank, local, barrier):
    """N > 1 side line: BASELINE configs[3] as written -- one 100M-record c4 capture split
    into `world` byte-balanced shares, each rank generating and editing only its own
    (strong scaling; the same code path as the verified c4 12.5M-record side line at N = 1).
    Whole-job records/s over the max-over-ranks time of K passes."""
    import torch
    import torch.distributed as dist
    total = 100_000_000
    share = make_share("c4", total, rank, world, seed=1)
    # each rank checks its share's first run against the sharded oracle (global record
    # numbers, the job's cache) when the share fits the checker's host memory: every rank
    # at N >= 4 (25M records, ~9 GB each)
    verify = not opt.no_verify and share[3] <= STRONG_VERIFY_MAX
    te, b, r, _, checked = run_workload("c4", share[3], 0, 2, seed=1, device=local, share=share, total=total,
                                        verify=verify)
    del share
    k = max(3, min(opt.steps, 20))
    byt = torch.tensor([r.bytes_in + r.bytes_out, r.packets, 1 if checked else 0, checked], dtype=torch.int64,
                       device="cuda")
    barrier()
    t0 = time.perf_counter()
    b.time(k)
    barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    dist.all_reduce(byt)
    b.close()
    te.close()
    sec = float(el.item()) / k
    return {"workload": f"{WORKLOADS['c4'][2]} over one {total}-record IMIX capture split into {world} "
                        "byte-balanced shares (BASELINE configs[3], strong scaling)",
            "records": int(byt[1].item()), "ms_per_pass": round(sec * 1e3, 4),
            "mpkt_s": round(int(byt[1].item()) / sec / 1e6, 1),
            "gbps_algorithmic": round(int(byt[0].item()) / sec / 1e9, 1),
            "frac_hbm_peak_per_gpu": round(int(byt[0].item()) / sec / 1e9 / world / HBM_PEAK_GBS, 4),
            "verified": int(byt[2].item()) == world, "verified_records": int(byt[3].item()),
            "note": "each rank's share checked against the oracle at its global record numbers"
                    if int(byt[2].item()) == world else
                    f"shares above {STRONG_VERIFY_MAX} records are not re-checked (host memory); the c4 code "
                    "path is checked at N=1"}


def e2e_line(opt):
    """the end_to_end line: host pcap bytes -> host output bytes through the pipelined path,
    run by `bench.py --e2e-child` in a process of its own (main() starts it)"""
    import tcpreplay_amd as TA
    n = opt.packets or DEFAULT_PACKETS[opt.workload]
    pcap = make_pcap(opt.workload, n, seed=1)
    # PCIe-inclusive rates (never `value`), host pcap bytes -> host output bytes,
    # through the pipelined path (chunks of whole records, H2D | edit | D2H on three
    # streams; median of 5 after a sizing run):
    #   pinned:   capture and output in page-locked memory (as bin/tcprewrite reads
    #             the file straight into it) -- the main figure;
    #   pageable: ordinary buffers, page-locked by the library for each call;
    #   one_shot: tcpedit_rewrite_pcap (device allocation, synchronous copies).
    te3 = TA.TcpEdit(WORKLOADS[opt.workload][2], device=0)
    src = bytearray(pcap)
    rc3, out3 = te3.rewrite_pipelined(src)  # sizes the device slots
    if not opt.no_verify:  # the pipelined path's output is the oracle's too
        check_output_bytes(pcap, WORKLOADS[opt.workload][2], None, out3)
    bound = te3.output_bound(src)
    pin_in, pin_out = TA.PinnedBuffer(len(pcap)), TA.PinnedBuffer(bound)
    pin_in.view[:] = pcap

    def e2e(si, so, reps=9):
        """median seconds of `reps` back-to-back runs, after 0.5 s of them: a fresh
        context's first ~0.2 s of pipelined runs copy at about half speed (3.8-4.1 ms
        against 2.09-2.14, every host-buffer kind alike, tools/e2e_host_ab.py)"""
        t_warm = time.perf_counter() + 0.5
        while time.perf_counter() < t_warm:
            te3.rewrite_pipelined(si, out=so)
        ts = []
        for _ in range(reps):
            t1 = time.perf_counter()
            rc, view = te3.rewrite_pipelined(si, out=so)
            ts.append(time.perf_counter() - t1)
            if rc != 0 or view != out3:
                raise RuntimeError("pipelined end-to-end run differs from its first run")
        return sorted(ts)[reps // 2]

    p_s = e2e(pin_in.view, pin_out.view)
    g_s = e2e(src, bytearray(bound))
    floor_ms = copy_floor(ctypes.addressof(ctypes.c_char.from_buffer(pin_in.view)), len(pcap),
                          ctypes.addressof(ctypes.c_char.from_buffer(pin_out.view)), len(out3))
    te3.rewrite(pcap)  # (its first call in a process allocates the one-shot buffers)
    one = []
    for _ in range(3):
        t1 = time.perf_counter()
        rc3, _out = te3.rewrite(pcap)
        one.append(time.perf_counter() - t1)
    pin_in.close()
    pin_out.close()
    te3.close()
    o_s = sorted(one)[1]

    def rate(sec, path):
        return {"mpkt_s": round(n / sec / 1e6, 2), "ms": round(sec * 1e3, 3),
                "gbps_in": round(len(pcap) / sec / 1e9, 2), "path": path}
    return dict(
        rate(p_s, "page-locked host capture -> byte-range chunks (the default: a tenth of the capture, "
                  "8-32 MiB; C/4 and C/2 first, halving last), H2D | window-mode edit (records found "
                  "on the device, chain verdict gathered on the device) | D2H on three streams -> "
                  "page-locked host output (median of 9 back-to-back runs after 0.5 s of them)"),
        copy_floor_ms=round(floor_ms, 3) if floor_ms else None,
        frac_of_copy_floor=round(floor_ms / (p_s * 1e3), 4) if floor_ms else None,
        copy_floor="this box's PCIe floor: the capture up and the output down at once, one copy each on "
                   "two streams, same page-locked buffers, no edit (median of 5)",
        pageable=rate(g_s, "the same from ordinary host buffers, page-locked per call (median of 9 "
                           "back-to-back runs after 0.5 s of them, timed after the page-locked block)"),
        one_shot=rate(o_s, "tcpedit_rewrite_pcap: device allocation, record index, synchronous "
                           "pageable copies (median of 3)"))


def extra_line(wl, steps, verify):
    """one secondary config's line (BASELINE configs[2..4] and the common tcprewrite lines),
    run by `bench.py --extra-child WL` in a process of its own (main() starts it): its first
    run checked against the oracle, then warm-up, kernel-only and pipeline timings"""
    n2 = DEFAULT_PACKETS[wl]
    te2, b2, r2, _, chk2 = run_workload(wl, n2, 0, 3, seed=11, device=0, verify=verify)
    k2 = max(20, steps // 50)
    b2.time(k2)  # (the first window after the oracle check runs up to 10 % slow: clocks/caches)
    # three alternating pipeline / kernel-only windows, the median of each (tools/extra_probe.py
    # XP_WINDOWS: one window in three still moved by 5-9 % on a box where the rest agreed)
    ps, ks = [], []
    for _ in range(3):
        ps.append(b2.time(k2))
        ks.append(b2.time_kernels(k2)[1])
    ms2, kms2 = sorted(ps)[1], sorted(ks)[1]
    ab = r2.bytes_in + r2.bytes_out
    line = {"workload": WORKLOADS[wl][3], "packets": n2, "pipeline_ms": round(ms2, 4),
            "kernel_ms": round(kms2, 4), "mpkt_s": round(n2 / (ms2 * 1e-3) / 1e6, 1),
            "gbps_algorithmic": round(ab / (ms2 * 1e-3) / 1e9, 1),
            "frac_hbm_peak": round(ab / (ms2 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "kernel_frac_hbm_peak": round(ab / (kms2 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "verified": chk2 == n2, "verified_records": chk2}
    b2.close()
    te2.close()
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--packets", type=int, default=0, help="records per GPU (default: the config's size)")
    ap.add_argument("--no-device-index", action="store_true", help="skip the device record index line")
    ap.add_argument("--no-packet-latency", action="store_true", help="skip the tcpedit_packet latency line")
    ap.add_argument("--extra", default="c3,c4,c5,c2x10,seed,hdr,vdel,efcs,macseed,mtu,fz,prep",
                    help="secondary configs measured at N=1 (comma list, '' = none)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU baseline budget (half 1 thread, "
                    "half --cpu-threads threads)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="threads of the multi-core CPU baseline "
                    "(default: the CPUs this process may run on, at most 16 -- the GPU box's CPU share)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive end-to-end rate")
    ap.add_argument("--e2e-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--extra-child", default="", help=argparse.SUPPRESS)
    ap.add_argument("--no-verify", action="store_true", help="skip the oracle check of every workload's "
                    "first run (on by default: the bench line is parity evidence)")
    ap.add_argument("--no-strong-side", action="store_true", help="N > 1: skip the BASELINE configs[3] line "
                    "(c4, 100M records split over the ranks)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: one --records-record capture split over the ranks (each rank "
                         "generates only its share); c4 defaults to BASELINE configs[3]'s 100M records")
    ap.add_argument("--records", type=int, default=0, help="--strong: the job's total records "
                    "(default 100M for c4, else the config's size)")
    opt = ap.parse_args()
    if opt.e2e_child:  # (main() of the parent process starts this)
        print(json.dumps(e2e_line(opt)), flush=True)
        return
    if opt.extra_child:  # (likewise)
        print(json.dumps(extra_line(opt.extra_child, opt.steps, not opt.no_verify)), flush=True)
        return
    if opt.strong:  # one big job: the per-config side lines measure other things
        opt.extra, opt.no_e2e, opt.no_cpu_baseline = "", True, True
        opt.no_device_index = opt.no_packet_latency = True

    import torch
    import torch.distributed as dist
    import tcpreplay_amd as TA
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    total = 0
    if opt.strong:
        total = opt.records or (100_000_000 if opt.workload == "c4" else DEFAULT_PACKETS[opt.workload])
        share = make_share(opt.workload, total, rank, world, seed=1)
        n = share[3]
        # verified when the share is small enough for the checker's host memory
        te, b, r, pcap, checked = run_workload(opt.workload, n, opt.steps, opt.warmup, seed=1, device=local,
                                               share=share, total=total,
                                               verify=not opt.no_verify and n <= STRONG_VERIFY_MAX)
        del share
    else:
        # N = 1: BASELINE configs[1] (1M x 64 B); N > 1: every rank the same 1M-record
        # workload (weak scaling, like with like)
        n = opt.packets or (PER_RANK_PACKETS.get(opt.workload, DEFAULT_PACKETS[opt.workload]) if world > 1
                            else DEFAULT_PACKETS[opt.workload])
        te, b, r, pcap, checked = run_workload(opt.workload, n, opt.steps, opt.warmup, seed=1 + rank,
                                               device=local, verify=not opt.no_verify)
    alg_bytes = r.bytes_in + r.bytes_out  # sum(16+caplen_in) + sum(16+caplen_out) per launch

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # untimed: the edit kernel's own mean duration (a hipEvent pair around it in every run;
    # those markers slow the pipeline slightly, so the timed loop below runs without them)
    _, kernel_ms = b.time_kernels(opt.steps)
    # the job's single counter reduction (RCCL all-reduce over xGMI at N > 1); the
    # tensor is built before the timed region, the collective runs inside it
    cnt = torch.tensor([r.packets * opt.steps, r.bytes_in * opt.steps, r.bytes_out * opt.steps,
                        r.written * opt.steps], dtype=torch.int64, device="cuda")
    barrier()
    t0 = time.perf_counter()
    # K back-to-back runs of the device pipeline (hipEvents on the library's launch stream)
    pipeline_ms = b.time(opt.steps)
    if world > 1:
        dist.all_reduce(cnt)
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    total_pkts = int(cnt[0].item())

    value = total_pkts / elapsed / 1e6
    # the dominant kernel's mean launch duration: when a run of the pipeline is that one
    # kernel (the wave lane with no tile left to the generic pass), the hipEvent pair around
    # the K back-to-back runs times exactly its K launches (rocprof agrees within ~1 %); a
    # hipEvent pair around every launch adds ~1.5 us of marker overhead to a 31 us kernel
    single = r.fast_kind == 2 and r.generic_tiles == 0
    dom_ms = pipeline_ms if single else kernel_ms
    achieved = alg_bytes / (dom_ms * 1e-3) / 1e9
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tfile) and not opt.strong:  # (profiled at the config's default size)
        try:
            tj = json.load(open(tfile))
            tkey = "c2x10" if opt.workload == "c2" and n == DEFAULT_PACKETS["c2x10"] else opt.workload
            traffic = tj.get(tkey, {}).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    # every rank checked its first run against the oracle (or did not): one flag, one count
    chk = torch.tensor([checked, 1 if checked else 0], dtype=torch.int64, device="cuda")
    if world > 1:
        dist.all_reduce(chk)
    if n == DEFAULT_PACKETS[opt.workload] or opt.strong:
        desc = WORKLOADS[opt.workload][3]
    else:
        desc = f"{WORKLOADS[opt.workload][2]} on {n} records per GPU of the {opt.workload} corpus " \
               f"({'HBM-resident weak-scaling shard; ' if world > 1 else ''}{WORKLOADS[opt.workload][3]})"
    result = {
        "metric": "Mpackets/s device-resident tcpedit rewrite+fixcsum",
        "value": round(value, 3),
        "unit": "Mpkt/s",
        "n_gpus": world,
        "steps": opt.steps,
        "warmup": opt.warmup,
        "ms_per_step": round(elapsed / opt.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "strong" if opt.strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (tcpreplay_amd.synth, seeded per rank)",
        "config": {"workload": (f"{WORKLOADS[opt.workload][2]} over one {total}-record capture split into "
                                f"{world} byte-balanced shares (BASELINE configs[3] for c4)")
                               if opt.strong else desc, "packets_per_gpu": n,
                   "tcpedit_args": WORKLOADS[opt.workload][2], "parallelism": f"shard{world}",
                   "global_records": total if opt.strong else n * world},
        "gbps_algorithmic": round((int(cnt[1].item()) + int(cnt[2].item())) / elapsed / 1e9, 2),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": TA.FAST_KERNELS.get(r.fast_kind, "te_edit_tiles"),
                     "kernel_ms": round(dom_ms, 5), "pipeline_ms": round(pipeline_ms, 5),
                     "kernel_ms_event_pairs": round(kernel_ms, 5),
                     "kernel_timing": "K back-to-back launches of the kernel alone between two hipEvents"
                                      if single else "a hipEvent pair around the kernel in each of K runs",
                     "alg_bytes_per_launch": alg_bytes},
        # parity on the bench's clock: each rank's first run == the oracle, byte for byte
        "verified": int(chk[1].item()) == world,
        "verified_records": int(chk[0].item()),
    }
    # the per-packet API (tcpedit_packet, as tcprewrite calls it once a record): one 64-byte
    # packet a call through the device (stage, edit, read back), beside the oracle's
    # per-record CPU time on the bulk workload
    if rank == 0 and not opt.no_packet_latency:
        from tcpreplay_amd import synth as S
        L = TA.load()
        f = L.tcpedit_debug_packet_latency
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        te1 = TA.TcpEdit(WORKLOADS[opt.workload][2])
        pkt = S.records(S.pcap_fixed(1, 64, seed=3))[0][4]
        us = ctypes.c_double()
        if f(te1._ctx, pkt, len(pkt), 2000, ctypes.byref(us)) == 0:
            result["packet_api"] = {"us_per_call": round(us.value, 2), "calls": 2000,
                                    "path": "tcpedit_packet through the resident device block: record and "
                                            "request in host-mapped memory, edited in LDS, response polled"}
        te1.close()
    # the record index built on the device (te_index.hip) from the HBM-resident image, in
    # place of the host walk: its build time, and the edit over the tiles it cut -- index +
    # edit is the device pipeline from the raw capture bytes
    if rank == 0 and not opt.no_device_index:
        applied, ims = b.index_device(iters=max(5, opt.steps // 20))
        if applied:
            pms2 = b.time(opt.steps)
            result["device_index"] = {
                "index_ms": round(ims, 5), "pipeline_ms": round(pms2, 5),
                "index_plus_pipeline_ms": round(ims + pms2, 5),
                "frac_hbm_peak_with_index": round(alg_bytes / ((ims + pms2) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "path": "windowed speculative record-boundary discovery + wave-lane tile cut on the device "
                        "(count, scan, write passes), then the edit over those tiles"}
        else:
            result["device_index"] = {"applied": False}
    # the window mode (tcpedit_batch_run_fused): the record discovery fused into the wave
    # lane -- one pass over the raw capture bytes plus the cross-window chain check, no
    # index passes and no tile list.  Its output is checked byte for byte against the
    # exact path's (itself checked against the oracle above).
    if rank == 0 and not opt.no_device_index:
        import numpy as np
        fms = b.time_fused(opt.steps)
        if fms is not None:
            ref = b.output_np()
            b.run_fused()
            same = b.fused_fallbacks == 0 and np.array_equal(ref, b.output_np())
            del ref
            result["fused"] = {
                "ms": round(fms, 5), "mpkt_s": round(r.packets / (fms * 1e-3) / 1e6, 1),
                "frac_hbm_peak": round(alg_bytes / (fms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "same_bytes_as_exact_path": bool(same),
                "path": "window mode: each wave stages 5 KiB windows of the raw capture, finds the records "
                        "(speculative boundary guesses checked along the chain), edits them in LDS and "
                        "stores them; te_win_check verifies the chain across windows"}
            if not same:
                raise RuntimeError("fused run differs from the exact path")
        else:
            result["fused"] = {"applied": False}
    b.close()
    te.close()
    if world > 1 and not opt.strong and not opt.no_strong_side:
        result["strong_c4"] = strong_side(opt, world, rank, local, barrier)

    if rank == 0 and world == 1:
        extra = {}
        for wl in [w for w in opt.extra.split(",") if w]:
            if wl == "prep":
                # tcpprep --port classification on C3's IMIX corpus:
                # tp_classify kernel, image and index resident in HBM; algorithmic bytes per
                # record = 12 (index) + 38 (Ethernet + IPv4 + L4 ports read) + 1/4 (cache entry)
                from tcpreplay_amd import tcpprep as TP
                n2 = 10_000_000
                tp = TP.TcpPrep(["--no-arg-comment", "--port"])
                prep_pcap = make_pcap("c3", n2, 11)
                kms2, ent = tp.time(prep_pcap, iters=max(5, opt.steps // 20))
                tp.close()
                # CPU baseline: the oracle (oracle/tcpprep_oracle.c, 1 thread) on the first
                # 1M records of the same capture, only the C call timed
                cpu_prep = None
                if not opt.no_cpu_baseline:
                    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests"))
                    import oracle_lib
                    from tcpreplay_amd import synth as _syn
                    sample = _syn.build_pcap(_syn.records(prep_pcap[:400_000_000])[:1_000_000])
                    t0 = time.perf_counter()
                    oracle_lib.tcpprep(sample, ["--no-arg-comment", "--port"])
                    cpu_s = time.perf_counter() - t0
                    cpu_prep = {"mpkt_s": round(1e6 / cpu_s / 1e6, 2), "cores": 1, "kind": "port",
                                "sample": "first 1M records of the same capture, oracle --port, 1 thread"}
                extra[wl] = {"workload": "tcpprep --port on IMIX 64/570/1514 7:4:1 (C3 corpus): v04 cache "
                                         "entries for every record", "packets": ent, "kernel_ms": round(kms2, 4),
                             "mpkt_s": round(ent / (kms2 * 1e-3) / 1e6, 1),
                             "gbps_algorithmic": round(ent * 50.25 / (kms2 * 1e-3) / 1e9, 1),
                             "cpu_baseline": cpu_prep}
                continue
            # each line in a child process of its own, as a tcprewrite run has the device (the
            # same runs measured 3-8 % slower inside this process after its other lines, the
            # pipeline column below the kernel-only one -- the cause was not isolated)
            import subprocess
            cmd = [sys.executable, os.path.abspath(__file__), "--extra-child", wl, "--steps", str(opt.steps)] + \
                (["--no-verify"] if opt.no_verify else [])
            cp = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
            if cp.returncode != 0:
                raise RuntimeError(f"extra line {wl} failed: {cp.stderr[-2000:]}")
            extra[wl] = json.loads(cp.stdout.strip().splitlines()[-1])
        if extra:
            result["extra_configs"] = extra
        if not opt.no_e2e:
            # PCIe-inclusive rates (never `value`): measured in a child process of their own
            # (e2e_line), as a tcprewrite run has the device to itself -- inside this process,
            # after the lines above, the same runs scattered over 2.3-2.9 ms against a steady
            # 2.1 in a fresh one (tools/e2e_host_ab.py, tools/gpu_e2e_bench_ab.sh)
            import subprocess
            cmd = [sys.executable, os.path.abspath(__file__), "--e2e-child", "--workload", opt.workload,
                   "--packets", str(n)] + (["--no-verify"] if opt.no_verify else [])
            cp = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
            if cp.returncode != 0:
                raise RuntimeError("end-to-end child failed: " + cp.stderr[-2000:])
            result["end_to_end"] = json.loads(cp.stdout.strip().splitlines()[-1])
        if not opt.no_cpu_baseline and opt.workload not in CACHED:
            wl_args = WORKLOADS[opt.workload][2]
            v1, runs1, el1, _ = cpu_baseline(pcap, wl_args, n, opt.cpu_seconds / 2)
            thr = opt.cpu_threads or min(16, len(os.sched_getaffinity(0)))
            v, runs, el, used = cpu_baseline(pcap, wl_args, n, opt.cpu_seconds / 2, thr)
            result["cpu_baseline"] = {
                "value": round(v, 3), "unit": "Mpkt/s", "cores": used, "kind": "port",
                "sample": f"{runs} passes of the oracle over the same {n}-record workload, split into {used} "
                          f"byte-balanced shards of whole records, one thread each ({el:.1f} s; in-memory, "
                          f"preallocated buffers, only the C call timed)",
                "single_thread": {"value": round(v1, 3), "cores": 1,
                                  "sample": f"{runs1} passes, 1 thread ({el1:.1f} s)"}}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
