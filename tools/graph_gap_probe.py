"""Probe: what a learner round costs beyond its kernels on the GPU box. Per iteration, on one stream: a HIP graph of
6 small dependent kernels, optionally with an event record / a cross-stream event wait / a second stream's kernel
around it, or the 6 kernels launched directly. Prints microseconds per iteration for each arrangement."""
import ctypes
import time

import torch


def main(size=1 << 16):
    dev = torch.device("cuda")
    print(f"-- kernels over {size} floats", flush=True)
    x = torch.zeros(size, device=dev)
    y = torch.zeros(1 << 16, device=dev)

    def six():
        for _ in range(6):
            x.add_(1.0)

    s1 = torch.cuda.Stream(device=dev)
    s2 = torch.cuda.Stream(device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s1):
        six()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s1):
            six()
    torch.cuda.synchronize()
    n = 400
    evs = [torch.cuda.Event() for _ in range(4)]

    def run(name, body):
        for i in range(20):
            body(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            body(i)
        torch.cuda.synchronize()
        print(f"{name:60s} {1e6 * (time.perf_counter() - t0) / n:8.1f} us/iter", flush=True)

    def direct(i):
        with torch.cuda.stream(s1):
            six()

    def graph(i):
        with torch.cuda.stream(s1):
            g.replay()

    def graph_rec(i):
        with torch.cuda.stream(s1):
            g.replay()
            evs[i & 3].record(s1)

    def graph_wait_done(i):  # wait on an event of s2 that completed long ago
        with torch.cuda.stream(s1):
            s1.wait_event(evs[0])
            g.replay()

    def graph_wait_s2(i):  # s2 runs one kernel per iteration, s1 waits for it, then replays
        with torch.cuda.stream(s2):
            y.add_(1.0)
            evs[i & 3].record(s2)
        with torch.cuda.stream(s1):
            s1.wait_event(evs[i & 3])
            g.replay()

    def direct_wait_s2(i):
        with torch.cuda.stream(s2):
            y.add_(1.0)
            evs[i & 3].record(s2)
        with torch.cuda.stream(s1):
            s1.wait_event(evs[i & 3])
            six()

    def ping_pong(i):  # s1 waits s2, s2 waits s1 (a dependency cycle per iteration)
        with torch.cuda.stream(s2):
            s2.wait_event(evs[(i + 1) & 3])
            y.add_(1.0)
            evs[i & 3].record(s2)
        with torch.cuda.stream(s1):
            s1.wait_event(evs[i & 3])
            x.add_(1.0)
            evs[(i + 2) & 3].record(s1)

    evs[0].record(s2)
    for e in evs:
        e.record(s1)
    torch.cuda.synchronize()
    run("6 kernels direct, one stream", direct)
    run("graph of 6 kernels, one stream", graph)
    run("graph + event record", graph_rec)
    run("wait on a completed event + graph", graph_wait_done)
    run("s2 kernel -> event -> s1 waits -> graph", graph_wait_s2)
    run("s2 kernel -> event -> s1 waits -> 6 kernels direct", direct_wait_s2)
    run("ping-pong s1 <-> s2, one kernel each", ping_pong)

    # the same cross-stream dependency through the HIP API directly: events with lighter release flags, and
    # stream memory operations (hipStreamWriteValue64 / hipStreamWaitValue64 on signal memory)
    hip = ctypes.CDLL("libamdhip64.so")
    vp = ctypes.c_void_p
    h1, h2 = vp(s1.cuda_stream), vp(s2.cuda_stream)
    for name, flags in (("DisableTiming", 0x2), ("DisableTiming|DisableSystemFence", 0x2 | 0x20000000),
                        ("DisableTiming|ReleaseToDevice", 0x2 | 0x40000000)):
        hev = [vp() for _ in range(4)]
        for e in hev:
            assert hip.hipEventCreateWithFlags(ctypes.byref(e), ctypes.c_uint(flags)) == 0

        def raw_wait(i, hev=hev):
            with torch.cuda.stream(s2):
                y.add_(1.0)
            assert hip.hipEventRecord(hev[i & 3], h2) == 0
            assert hip.hipStreamWaitEvent(h1, hev[i & 3], ctypes.c_uint(0)) == 0
            with torch.cuda.stream(s1):
                g.replay()

        run(f"s2 kernel -> hipEvent({name}) -> s1 waits -> graph", raw_wait)
    sig = vp()
    assert hip.hipExtMallocWithFlags(ctypes.byref(sig), ctypes.c_size_t(8), ctypes.c_uint(0x2)) == 0
    assert hip.hipMemset(sig, 0, ctypes.c_size_t(8)) == 0
    torch.cuda.synchronize()
    cnt = [0]

    def value_wait(i):
        cnt[0] += 1
        with torch.cuda.stream(s2):
            y.add_(1.0)
        assert hip.hipStreamWriteValue64(h2, sig, ctypes.c_uint64(cnt[0]), ctypes.c_uint(0)) == 0
        assert hip.hipStreamWaitValue64(h1, sig, ctypes.c_uint64(cnt[0]), ctypes.c_uint(0),
                                        ctypes.c_uint64(0xFFFFFFFFFFFFFFFF)) == 0
        with torch.cuda.stream(s1):
            g.replay()

    run("s2 kernel -> hipStreamWriteValue64 -> s1 hipStreamWaitValue64 -> graph", value_wait)


if __name__ == "__main__":
    main()
    main(1 << 23)  # ~10-us kernels: the host is far ahead, so only GPU-side costs remain
