"""PCIe copy rates by piece size and stream count (diagnostic): 80 MB from/to page-locked
host memory as one copy or as pieces, on 1 or 2 streams per direction, each direction
alone and both at once -- what the pipeline's chunked copies can reach."""
import ctypes
import statistics
import time

hip = ctypes.CDLL("libamdhip64.so")
N = 80 << 20


def alloc_host(n):
    p = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(n), 0) == 0
    return p.value


def alloc_dev(n):
    p = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(n)) == 0
    return p.value


def stream():
    s = ctypes.c_void_p()
    hip.hipStreamCreateWithFlags(ctypes.byref(s), 1)
    return s


hin, hout = alloc_host(N), alloc_host(N)
din, dout = alloc_dev(N), alloc_dev(N)
ctypes.memset(hin, 1, N)
up = [stream(), stream()]
down = [stream(), stream()]


def run(piece, nup, ndown, reps=7):
    ts = []
    for _ in range(reps):
        hip.hipDeviceSynchronize()
        t0 = time.perf_counter()
        k = 0
        for off in range(0, N, piece):
            n = min(piece, N - off)
            if nup:
                hip.hipMemcpyAsync(ctypes.c_void_p(din + off), ctypes.c_void_p(hin + off), ctypes.c_size_t(n), 1,
                                   up[k % nup])
            if ndown:
                hip.hipMemcpyAsync(ctypes.c_void_p(hout + off), ctypes.c_void_p(dout + off), ctypes.c_size_t(n), 2,
                                   down[k % ndown])
            k += 1
        hip.hipDeviceSynchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


for piece in (N, 16 << 20, 8 << 20, 4 << 20, 2 << 20):
    for nup, ndown in ((1, 0), (0, 1), (2, 0), (0, 2), (1, 1), (2, 2), (1, 2)):
        t = run(piece, nup, ndown)
        moved = N * ((nup > 0) + (ndown > 0))
        print(f"piece {piece >> 20:3d} MiB up x{nup} down x{ndown}: {t * 1e3:6.3f} ms  {moved / t / 1e9:6.1f} GB/s",
              flush=True)
