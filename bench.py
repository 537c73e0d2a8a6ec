#!/usr/bin/env python3
"""bench.py — device-resident CRC-32 (Ethernet FCS) throughput on MI355X.

Metric (BASELINE.json): GiB/s of CRC-32 over device-resident 1500-byte frames,
with the fraction of the HBM3E read roofline.  One "step" = one
lnx_crc32_batch call over the rank's whole frame batch (inputs already in HBM).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME] [--op OP]

--op crc32 (default, the BASELINE metric) | fcs_append (lnx_fcs_append_batch: TX FCS
append in place on 1496-B frames in 1536-B ring slots, lengths reset each step) | tx_finish (lnx_tx_finish_batch:
checksum generate + pad + FCS of the same UDP/IPv4 frames in one read) | fcs_verify (lnx_fcs_verify_batch,
residue check of the same frames) | sum16 (lnx_sum16_batch: RFC 791 checksum of
every frame as one segment, random pseudo-header seeds) | ingress
(lnx_ingress_verify_batch: the frames get Ethernet/IPv4/UDP headers written in
place, so every frame takes the full header-sum + UDP-sum path).

N=1 runs BASELINE configs[1] (1 M x 1500 B) and, beside `value`, a "slice16m"
sub-measurement: the same kernel over 16 M x 1500 B, the per-GPU slice the
N>1 runs use, so the driver's scaling series has an equal-work N=1 point.  For
N>1 (launched by torch.distributed.run, one rank per GPU) every rank owns its
own contiguous slice of configs[4] (128 M x 1500 B over 8 GPUs = 16 M frames
per GPU); frames are partitioned by index with no data-path collective (weak
scaling).  The barrier / MAX-over-ranks timing runs over a gloo process group
(host-side clock only): the path needs no RCCL, so none is initialised.

Rank 0 prints ONE JSON line.  Extra fields: "roofline" (dominant kernel,
HIP-event timed on its launch stream), "cpu_baseline" (the C oracle on the
box's host cores, bounded sample, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md
FRAME_BYTES = 1500


def shard_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous frame-index slice [lo, hi) of rank `rank`."""
    per = (n_total + world - 1) // world
    lo = min(rank * per, n_total)
    hi = min(lo + per, n_total)
    return lo, hi


def workload_spec(name: str, world: int):
    """(frames on this rank, frame length or None for zipf, description)."""
    if name == "auto":
        name = "mtu1500" if world == 1 else "mtu1500_x8"
    if name == "mtu1500":
        return name, 1 << 20, 1500, "configs[1]: 1M x 1500B device-resident, 1 GPU"
    if name == "mtu1500_x8":
        return name, (1 << 27) // 8, 1500, "configs[4]: 128M x 1500B over 8 GPUs (16M per GPU), per-GPU partition"
    if name == "jumbo9000":
        return name, 1 << 20, 9000, "configs[2]: 1M x 9000B device-resident, 1 GPU"
    if name == "zipf64_1500":
        return name, 1 << 24, None, "configs[3]: 16M mixed 64-1500B (Zipf s=1), 1 GPU"
    raise SystemExit(f"unknown workload {name}")


def go_maxprocs() -> tuple[int, str]:
    """The thread count Go's runtime would default GOMAXPROCS to on this host
    (go1.25+, the reference's CI runs go1.26): the CPUs this process may run
    on (sched_getaffinity, what `nproc` prints), capped by a cgroup v2 CPU
    bandwidth limit when one is set (rounded up, at least 2)."""
    n = len(os.sched_getaffinity(0))
    rule = f"sched_getaffinity {n}"
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if quota != "max":
            lim = max(2, -(-int(quota) // int(period)))
            rule += f", cgroup cpu.max {quota}/{period} -> {lim}"
            n = min(n, lim)
    except (OSError, ValueError):
        pass
    return n, rule


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(d_bytes, off_np, frame_len, budget_s: float = 10.0, threads: int | None = None, op: str = "crc32"):
    """Time the C oracle on a bounded sample of the same frames: for CRC-32 the
    restatement of Go hash/crc32 as its amd64 build runs ethernet/crc.go:19-21
    (archUpdateIEEE: PCLMULQDQ folding for >= 64 bytes, slicing-by-8 tail; the
    plain slicing-by-8 form is reported beside it), for --op sum16 the
    crc.go:52-59 restatement."""
    from oracle import oracle as O
    rule = "given"
    if threads is None:
        threads, rule = go_maxprocs()
    if op == "search":
        # the C restatement of ethernet/crc.go:28-47 (crc32.Update per byte), one thread
        nsamp = min(len(off_np) - 1, 256)
        caps = [d_bytes[int(off_np[i]):int(off_np[i + 1])].cpu().numpy().tobytes() for i in range(nsamp)]
        sb = sum(len(c) for c in caps)
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget_s / 2:
            for c in caps:
                O.c_crc32_search(c, 0)
            reps += 1
        el = time.perf_counter() - t0
        return {"value": round(reps * sb / el / 2**30, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
                "cpu_model": cpu_model(),
                "sample": f"{nsamp} captures x {frame_len} B; C restatement of ethernet/crc.go CRC32Search "
                          "(one crc32.Update per byte), NOT lneto's Go binary"}
    if op == "sum16":
        threads = 1  # the C oracle's segment sum is single-threaded
    nsamp = min(len(off_np) - 1, 1 << 16)
    sample_bytes = int(off_np[nsamp] - off_np[0])
    host = d_bytes[int(off_np[0]):int(off_np[nsamp])].cpu().numpy()
    off_s = (off_np[:nsamp + 1] - off_np[0]).astype(np.uint64)
    res = {}
    lens_s = np.diff(off_s).astype(np.uint32)
    amd64 = op != "sum16" and O.has_clmul()

    def run(t, fast):
        if op == "sum16":
            O.sum16_segments(host, off_s[:-1], lens_s, None)
        else:
            O.crc32_frames(host, off_s, threads=t, amd64=fast)

    forms = [(t, amd64) for t in sorted({1, threads})] + ([(threads, False)] if amd64 else [])
    slot = budget_s / (2 * max(1, len(forms) - 1))
    for t, fast in forms:
        run(t, fast)  # warm
        reps, t0 = 0, time.perf_counter()
        while True:
            run(t, fast)
            reps += 1
            el = time.perf_counter() - t0
            if el >= slot:
                break
        res[(t, fast)] = reps * sample_bytes / el / 2**30
    out = {
        "value": round(res[(threads, amd64)], 3), "unit": "GiB/s", "cores": threads, "kind": "port",
        "cpu_model": cpu_model(), "threads_rule": "GOMAXPROCS default: " + rule,
        "value_1core": round(res[(1, amd64)], 3),
        "sample": f"{nsamp} frames x {frame_len or 'zipf'} B ({sample_bytes/1e6:.0f} MB) of the same synthetic batch, "
                  f"repeated for ~{slot:.0f}s per form; " + (
                      "C restatement of lneto crc.go PayloadSum16" if op == "sum16" else
                      "C restatement of Go hash/crc32 as its amd64 build runs it (PCLMULQDQ folding, "
                      "slicing-by-8 tail)" if amd64 else "C restatement of Go hash/crc32 (slicing-by-8)") +
                  ", NOT lneto's Go binary (no Go toolchain on the box)",
    }
    if amd64:
        out["value_slicing8"] = round(res[(threads, False)], 3)
    return out


def rx_ring_bench(args, L, synth, torch, dev, world):
    """PCIe-inclusive receive path: frames
    (incl. their LE FCS) sit in the ring's pinned host slots as a NIC would
    leave them; one step = lnx_rx_ring_ingress over all of them: H2D, FCS
    verify, receive-path verdicts, D2H, pipelined over --ring-depth HIP
    streams.  --workload mtu1500: 1 M x 1500 B (slots nearly full: whole-slot
    copies); zipf64_1500: 1 M frames of the Zipf mix (mean ~246 B) in the same
    1536-B slots (packed on the host: PCIe carries the frames and their
    offsets).  Host wall clock per step; never the headline `value`."""
    if world != 1:
        raise SystemExit("--op rx_ring runs on one GPU")
    n, cap = 1 << 20, 1536
    zipf = args.workload == "zipf64_1500"
    if zipf:
        lens_np = synth.zipf_lengths(n).astype(np.int64)
    else:
        lens_np = np.full(n, FRAME_BYTES, dtype=np.int64)
    off_np = synth.offsets_from_lengths(lens_np).astype(np.int64)
    d = synth.bytes_torch(int(off_np[-1]), dev)
    d_off = torch.from_numpy(off_np).to(dev)
    # the last 4 bytes of every frame: the LE FCS of the rest
    starts = d_off[:-1].contiguous()
    lens = torch.from_numpy((lens_np - 4).astype(np.int32)).to(dev)
    fcs = L.crc32_segments(d, starts, lens)
    pos = (starts + lens.to(torch.int64)).unsqueeze(1) + torch.arange(4, device=dev)
    d[pos.reshape(-1)] = fcs.view(torch.uint8).view(-1)
    host = d.cpu().numpy()
    del d, pos
    ring = L.RxRing(n, slot_cap=cap, batch_slots=args.ring_batch, depth=args.ring_depth)
    zero_copy = not args.ring_copy
    try:
        ring.set_zero_copy(zero_copy)
        # slot i = frame i at offset 0
        if zipf:
            slots = ring.slots
            for i in range(n):
                slots[i, :lens_np[i]] = host[off_np[i]:off_np[i + 1]]
        else:
            ring.slots[:, :FRAME_BYTES] = host.reshape(n, FRAME_BYTES)
        ring.lengths[:] = lens_np.astype(np.uint32)
        for _ in range(max(args.warmup, 1)):
            ok, verdict = ring.ingress(0, n)
        assert ok.all(), "FCS verify failed on valid frames"
        t0 = time.perf_counter()
        for _ in range(args.steps):
            ring.ingress(0, n)
        el = (time.perf_counter() - t0) / args.steps
    finally:
        ring.close()
    nbytes = int(off_np[-1])
    batches = -(-n // args.ring_batch)
    fill = nbytes / (n * cap)
    packed = fill < 0.9  # the ring's rule (rx_ring.hip lnx_rx_ring_ingress)
    if zero_copy:  # the kernel reads the frame bytes in place; DMA moves only the lengths
        h2d, copy = nbytes + 4 * n, "zero copy (kernel reads the pinned slots; lengths by DMA)"
    else:
        h2d = nbytes + 8 * (n + batches) if packed else n * cap + 4 * n
        copy = "packed (frames + offsets)" if packed else "whole slots"
    out = {
        "metric": "GiB/s receive ring, PCIe-inclusive (pinned slots -> FCS verify + ingress verdicts -> D2H)",
        "value": round(nbytes / el / 2**30, 2), "unit": "GiB/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(el * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": f"synthetic {'Zipf 64-1500 B' if zipf else '1500-byte'} frames with valid FCS in {cap}-byte slots",
        "config": {"workload": f"1M {'Zipf-mix' if zipf else 'x 1500 B'} frames in host memory", "frames": n,
                   "frame_bytes": nbytes, "slot_cap": cap, "slot_fill": round(fill, 4),
                   "copy": copy,
                   "pcie_bytes_per_step": h2d, "pcie_d2h_bytes_per_step": 2 * n,
                   "pcie_bytes_per_frame_byte": round(h2d / nbytes, 4),
                   "depth": args.ring_depth, "batch_slots": args.ring_batch, "kernel": L.version()},
    }
    print(json.dumps(out), flush=True)


def _udp4_frames(synth, n, cap, lens):
    """n UDP/IPv4 Ethernet frames of lens[i] bytes, frame i = rows[i, :lens[i]]
    of a pageable (n, cap) array: random payload, headers the TX generate and
    the receive verdicts accept (EtherType 0x0800, IHL 5, DF, TTL 64, UDP)."""
    rows = synth.bytes_np(n * cap, seed=synth.SEED).reshape(n, cap)
    rows[:, 0:6] = (0x02, 0x00, 0x00, 0x00, 0x00, 0x01)
    rows[:, 6:12] = (0x02, 0x00, 0x00, 0x00, 0x00, 0x02)
    rows[:, 12:16] = (0x08, 0x00, 0x45, 0x00)
    ip_len = (lens - 14).astype(np.uint32)
    rows[:, 16] = (ip_len >> 8) & 0xFF
    rows[:, 17] = ip_len & 0xFF
    rows[:, 20:24] = (0x40, 0x00, 64, 17)
    rows[:, 24:26] = 0
    rows[:, 26:34] = (10, 0, 0, 1, 10, 0, 0, 2)
    udp_len = (lens - 34).astype(np.uint32)
    rows[:, 38] = (udp_len >> 8) & 0xFF
    rows[:, 39] = udp_len & 0xFF
    rows[:, 40:42] = 0
    return rows


def _udp4_device(L, torch, d_bytes, starts, lens, fcs: bool, chunk: int = 1 << 20):
    """Valid UDP/IPv4 frames in place on the device: frame i = d_bytes[starts[i] :
    starts[i] + lens[i]] (int64 / int64 device tensors) gets an Ethernet + IPv4 +
    UDP header whose length fields cover the frame (without its last 4 bytes
    when `fcs`), its IPv4 header and UDP checksums (lnx_tx_checksum_batch) and,
    when `fcs`, its LE FCS in the last 4 bytes (lnx_crc32_segments), so the
    receive check accepts every frame.  Headers in chunks of `chunk` frames
    (an index tensor of 42 entries per frame)."""
    dev = d_bytes.device
    body = lens - 4 if fcs else lens
    hdr = torch.tensor(list(bytes.fromhex("c0ffee00dead4e8b3af9fb6b0800") + bytes([0x45, 0, 0, 0])
                            + bytes.fromhex("123440004011000" + "0c0a80a01c0a80a02")
                            + bytes.fromhex("14e9003500000000")), dtype=torch.uint8, device=dev)
    col = torch.arange(42, device=dev)
    for a in range(0, starts.numel(), chunk):
        st, bl = starts[a:a + chunk], body[a:a + chunk]
        h = hdr.repeat(st.numel(), 1)
        ip, udp = bl - 14, bl - 34
        h[:, 16], h[:, 17] = (ip >> 8).to(torch.uint8), (ip & 255).to(torch.uint8)
        h[:, 38], h[:, 39] = (udp >> 8).to(torch.uint8), (udp & 255).to(torch.uint8)
        d_bytes[(st[:, None] + col).reshape(-1)] = h.reshape(-1)
    st = L.tx_checksum_batch(d_bytes, starts, body.to(torch.int32))
    assert int(st.max()) == 0, "UDP/IPv4 frame construction"
    if fcs:
        c = L.crc32_segments(d_bytes, starts, body.to(torch.int32))
        for a in range(0, starts.numel(), chunk):
            pos = (starts[a:a + chunk] + body[a:a + chunk])[:, None] + torch.arange(4, device=dev)
            d_bytes[pos.reshape(-1)] = c[a:a + chunk].view(torch.uint8).view(-1)


def packets_bench(args, L, synth, torch, dev, world):
    """The netdev batch boundary end to end (x/netdev/interface.go:85-89,
    DESIGN.md §4): per-frame pageable host buffers, as a Go stack hands them
    over.  egress_packets: lnx_egress_packets with LNX_TX_CHECKSUM | LNX_TX_FCS
    (gather into pinned staging, H2D, TX checksum generate + padding + FCS
    append, D2H, scatter back into the buffers); ingress_packets:
    lnx_ingress_packets (gather, H2D, FCS verify + receive verdicts, D2H).
    1 M frames, --workload mtu1500 (1500 B on the wire) or zipf64_1500.
    Host wall clock per step; never the headline `value`."""
    if world != 1:
        raise SystemExit(f"--op {args.op} runs on one GPU")
    n, cap = 1 << 20, 1536
    zipf = args.workload == "zipf64_1500"
    wire = synth.zipf_lengths(n).astype(np.int64) if zipf else np.full(n, FRAME_BYTES, dtype=np.int64)
    rows = _udp4_frames(synth, n, cap, wire)
    slot_bufs = args.bufs == "slots"
    if slot_bufs:
        # RunnerConfig.Buffers carved from the ring's slots (x/netdev/runner.go:92-94): the
        # kernels read (egress: patch) the frames in place
        ring = L.RxRing(n, slot_cap=cap, batch_slots=args.ring_batch, depth=args.ring_depth)
        ring.slots[:] = rows
        del rows
        rows = ring.slots
    else:
        ring = L.RxRing(args.ring_batch, slot_cap=cap,  # (the packet calls stage through the ring)
                        batch_slots=args.ring_batch, depth=args.ring_depth)
    ring.set_zero_copy(not args.ring_copy)
    ptrs = (rows.ctypes.data + cap * np.arange(n, dtype=np.uint64)).astype(np.uint64)
    status = np.zeros(n, dtype=np.uint8)
    verdict = np.zeros(n, dtype=np.uint8)
    try:
        if args.op == "egress_packets":
            sizes0 = (wire - 4).astype(np.uint32)  # the stack's frame; the device adds the FCS
            lens = sizes0.copy()

            def step():
                lens[:] = sizes0
                rc = L.lib.lnx_egress_packets(ring._h, ptrs.ctypes.data, lens.ctypes.data, n, 0, cap,
                                              L.TX_CHECKSUM | L.TX_FCS, status.ctypes.data)
                if rc != 0:
                    raise L.LnetoError(f"lnx_egress_packets: {rc}")
            step()
            assert (lens == wire.astype(np.uint32)).all() and (status == 0).all(), "egress: unexpected lengths/status"
            room = np.maximum(sizes0.astype(np.int64), 60) + 4
            zc = ring.stats()["zero_copy_frames"]
            if zc:
                assert zc == n, f"egress: {zc} of {n} frames zero-copy"
                h2d = 2 * int(sizes0.sum()) + 12 * n  # both kernels read the frame in place
                d2h = 6 * n  # (+ the in-place header / FCS stores)
                what = "slot buffers in place: TX checksum generate + pad + FCS append on the pinned slots"
            else:
                h2d = int(room.sum()) + 12 * n
                d2h = int(room.sum()) + 6 * n
                what = "gather -> H2D -> TX checksum generate + pad + FCS append -> D2H -> scatter"
        else:
            # frames already finished by the transmit path: run egress once to give them checksums + FCS
            sizes0 = (wire - 4).astype(np.uint32)
            lens = sizes0.copy()
            rc = L.lib.lnx_egress_packets(ring._h, ptrs.ctypes.data, lens.ctypes.data, n, 0, cap,
                                          L.TX_CHECKSUM | L.TX_FCS, status.ctypes.data)
            assert rc == 0 and (status == 0).all()
            lens = wire.astype(np.uint32)

            def step():
                rc = L.lib.lnx_ingress_packets(ring._h, ptrs.ctypes.data, lens.ctypes.data, n, 0, 0,
                                               status.ctypes.data, verdict.ctypes.data)
                if rc != 0:
                    raise L.LnetoError(f"lnx_ingress_packets: {rc}")
            z0 = ring.stats()["zero_copy_frames"]
            step()
            assert (status == 1).all() and (verdict == 0).all(), "ingress: valid frames not accepted"
            d2h = 2 * n
            if ring.stats()["zero_copy_frames"] - z0 == n:
                h2d = int(wire.sum()) + 12 * n
                what = "slot buffers in place: frame table H2D -> FCS verify + receive verdicts -> D2H"
            else:
                h2d = int(wire.sum()) + 8 * (n + -(-n // args.ring_batch))
                what = "gather -> H2D -> FCS verify + receive verdicts -> D2H"
        for _ in range(max(args.warmup, 1) - 1):
            step()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        el = (time.perf_counter() - t0) / args.steps
    finally:
        ring.close()
    nbytes = int(wire.sum())
    out = {
        "metric": f"GiB/s {args.op} ({'ring slot buffers' if slot_bufs else 'per-frame pageable buffers'}: {what})",
        "value": round(nbytes / el / 2**30, 2), "unit": "GiB/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(el * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": f"synthetic UDP/IPv4 {'Zipf 64-1500 B' if zipf else '1500-byte'} frames (on the wire), "
                f"one {'pinned ring slot' if slot_bufs else 'pageable'} {cap}-byte buffer each",
        "config": {"workload": f"1M {'Zipf-mix' if zipf else 'x 1500 B'} frames in host memory", "frames": n,
                   "frame_bytes": nbytes, "pcie_h2d_bytes_per_step": h2d, "pcie_d2h_bytes_per_step": d2h,
                   "mpps": round(n / el / 1e6, 2), "depth": args.ring_depth, "batch_slots": args.ring_batch,
                   "kernel": L.version()},
    }
    print(json.dumps(out), flush=True)


def slice16m_bench(L, synth, torch, dev, steps: int = 10, warmup: int = 3):
    """configs[4]'s per-GPU slice (16 M x 1500 B, 24 GB) on this one GPU: the
    per-rank work of every N>1 run, so value_N / (N * slice16m) compares equal
    launch sizes.  Reported beside `value`, never as it."""
    n, flen = (1 << 27) // 8, FRAME_BYTES
    d = synth.bytes_torch(n * flen, dev, seed=synth.SEED)
    o = torch.arange(n + 1, dtype=torch.int64, device=dev) * flen
    c = torch.empty(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    for _ in range(warmup):
        L.crc32_batch(d, o, out=c, stream=s)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        L.crc32_batch(d, o, out=c, stream=s)
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / steps
    del d, o, c
    torch.cuda.empty_cache()
    return {"value": round(n * flen / el / 2**30, 2), "unit": "GiB/s", "ms_per_step": round(el * 1e3, 4),
            "frames": n, "frame_bytes": flen, "steps": steps,
            "frac_hbm": round(n * flen / el / 1e9 / HBM_PEAK_GBS, 4),
            "note": "configs[4] per-GPU slice on one GPU: the equal-work N=1 point of the scaling series"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="auto",
                    choices=["auto", "mtu1500", "mtu1500_x8", "jumbo9000", "zipf64_1500"])
    ap.add_argument("--op", default="crc32",
                    choices=["crc32", "fcs_verify", "fcs_append", "tx_finish", "sum16", "ingress", "rx_ring", "search",
                             "tx_checksum", "egress_packets", "ingress_packets", "rx_verify", "pcap"])
    ap.add_argument("--short-frames", action="store_true",
                    help="--op crc32 / fcs_verify through lnx_*_batch_ex(LNX_BATCH_SHORT_FRAMES): the staged "
                         "lane-stream kernel the caller picks for a short-frame mix (DESIGN.md §3.9)")
    ap.add_argument("--ring-depth", type=int, default=3, help="--op rx_ring: pipeline stages")
    ap.add_argument("--ring-batch", type=int, default=65536, help="--op rx_ring: slots per stage batch")
    ap.add_argument("--ring-copy", action="store_true",
                    help="--op rx_ring / *_packets: copy frames through staging (lnx_rx_ring_set_zero_copy(0))")
    ap.add_argument("--bufs", choices=["own", "slots"], default="own",
                    help="--op *_packets: pageable buffers of the caller, or views of the ring's slots")
    ap.add_argument("--prewarm-s", type=float, default=0.5,
                    help="untimed launches for this long before the W warmup steps (GPU clock ramp)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-slice16m", action="store_true", help="skip the 16 M-frame equal-work sub-measurement")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--with-copies", action="store_true", help="also time pinned H2D+kernel+D2H")
    ap.add_argument("--verify", action="store_true", help="spot-check results against the oracle")
    args = ap.parse_args()

    import torch
    import lneto_amd as L
    from lneto_amd import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        if world == 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run (one rank per GPU)")
    # LNETO_BENCH_SHARE_GPU=1 (rehearsal on a one-GPU box only): every rank
    # uses cuda:0.  LNETO_BENCH_CPU_RANKS=1 (CPU test of the N>1 control flow,
    # tests/test_multi_gloo.py): no GPU at all, the step is the host C path.
    share = os.environ.get("LNETO_BENCH_SHARE_GPU") == "1"
    cpu_ranks = os.environ.get("LNETO_BENCH_CPU_RANKS") == "1"
    gpu = 0 if share else local_rank
    if cpu_ranks:
        dev = torch.device("cpu")
    else:
        torch.cuda.set_device(gpu)
        dev = torch.device("cuda", gpu)
    dist = None
    if world > 1:
        # The barrier and the 2-float max-over-ranks are host-side: gloo.  The
        # path has no exchange step, so no RCCL communicator
        # is created (an 8-rank RCCL init would be a failure point unrelated to it).
        import torch.distributed as dist
        dist.init_process_group("gloo")
    cdev = torch.device("cpu")  # device of the timing tensors (gloo)

    if args.op == "rx_ring":
        return rx_ring_bench(args, L, synth, torch, dev, world)
    if args.op in ("egress_packets", "ingress_packets"):
        return packets_bench(args, L, synth, torch, dev, world)

    wname, n_rank, flen, desc = workload_spec(args.workload, world)
    if cpu_ranks:
        if args.op != "crc32":
            raise SystemExit("LNETO_BENCH_CPU_RANKS runs --op crc32 only")
        # the control flow of an N-rank run on host cores: a small batch, the
        # library's host CRC per frame (no GPU, no oracle)
        n_rank = int(os.environ.get("LNETO_BENCH_CPU_FRAMES", "512"))
        desc += f" [CPU rehearsal: {n_rank} frames per rank, host lnx_crc32, no GPU]"
    # Frame index slice of this rank within the global batch (weak scaling:
    # the global batch grows with N, every rank owns n_rank frames).
    n_total = n_rank * world
    lo, hi = shard_range(n_total, world, rank)
    n_local = hi - lo
    if flen is None:
        lens = synth.zipf_lengths(n_local, seed=synth.ZIPF_SEED + rank)
        off_np = synth.offsets_from_lengths(lens)
    else:
        off_np = synth.fixed_offsets(n_local, flen)
    nbytes = int(off_np[-1])
    zipf_slots = False  # --op tx_finish on the Zipf mix: frames in slots, off_np the slot grid
    d_bytes = synth.bytes_torch(nbytes, dev, seed=synth.SEED + lo * 0x10001)
    d_off = torch.from_numpy(off_np.astype(np.int64)).to(dev)
    d_crc = torch.empty(n_local, dtype=torch.int32, device=dev)
    stream = None if cpu_ranks else torch.cuda.current_stream(dev)

    def sync():
        if not cpu_ranks:
            torch.cuda.synchronize(dev)
    if args.op == "sum16":
        d_seg = d_off[:-1].contiguous()
        d_len = (d_off[1:] - d_off[:-1]).to(torch.int32)
        d_seed = torch.randint(0, 1 << 20, (n_local,), dtype=torch.int32, device=dev)
        d_sum = torch.empty(n_local, dtype=torch.int16, device=dev)
    elif args.op == "fcs_verify":
        d_ok = torch.empty(n_local, dtype=torch.uint8, device=dev)
    elif args.op == "tx_finish" and flen is None:
        # the transmit tail on the Zipf mix: frame i (its wire length less the
        # FCS, >= 60 B: no padding) in a 1536-byte slot, valid UDP/IPv4 headers
        cap = 1536
        n_slots = n_local
        wire = torch.from_numpy(lens.astype(np.int64)).to(dev)
        d_bytes = synth.bytes_torch(n_slots * cap, dev, seed=synth.SEED + lo * 0x10001)
        d_start = torch.arange(n_slots, dtype=torch.int64, device=dev) * cap
        _udp4_device(L, torch, d_bytes, d_start, wire - 4, fcs=False)
        d_len0 = (wire - 4).to(torch.int32)
        d_len = d_len0.clone()
        d_status = torch.empty(n_slots, dtype=torch.uint8, device=dev)
        nbytes = int((wire - 4).sum())
        zipf_slots = True
    elif args.op == "tx_finish":
        # the transmit tail in one read (lnx_tx_finish_batch): UDP/IPv4 frames of
        # flen - 4 bytes in CAP-byte slots get their length fields and checksums
        # (idempotent) and their LE FCS in place; the lengths are restored first
        # every step (a 4-byte-per-frame device copy, timed)
        cap = 1536
        n_slots = n_local
        d_bytes = synth.bytes_torch(n_slots * cap, dev, seed=synth.SEED + lo * 0x10001)
        fr = d_bytes.view(n_slots, cap)
        hdr = bytes.fromhex("c0ffee00dead4e8b3af9fb6b0800") + bytes([0x45, 0]) + (flen - 18).to_bytes(2, "big") \
            + bytes.fromhex("12344000401100 00c0a80a01c0a80a02".replace(" ", "")) \
            + bytes.fromhex("14e90035") + (flen - 38).to_bytes(2, "big")
        fr[:, : len(hdr)] = torch.tensor(list(hdr), dtype=torch.uint8, device=dev)
        nbytes = n_slots * (flen - 4)
        d_start = torch.arange(n_slots, dtype=torch.int64, device=dev) * cap
        d_len0 = torch.full((n_slots,), flen - 4, dtype=torch.int32, device=dev)
        d_len = d_len0.clone()
        d_status = torch.empty(n_slots, dtype=torch.uint8, device=dev)
        off_np = (np.arange(n_slots + 1, dtype=np.int64) * cap)
    elif args.op == "fcs_append":
        # TX path (internet/stack-ethernet.go:200-214): frames of flen - 4 bytes
        # in slots of CAP bytes get their LE FCS appended in place; the step
        # restores the lengths first (a 4-byte-per-frame device copy, timed)
        if flen is None:
            raise SystemExit("--op fcs_append needs fixed-size frames")
        cap = 1536
        n_slots = n_local
        d_bytes = synth.bytes_torch(n_slots * cap, dev, seed=synth.SEED + lo * 0x10001)
        nbytes = n_slots * (flen - 4)
        d_start = torch.arange(n_slots, dtype=torch.int64, device=dev) * cap
        d_len0 = torch.full((n_slots,), flen - 4, dtype=torch.int32, device=dev)
        d_len = d_len0.clone()
        d_status = torch.empty(n_slots, dtype=torch.uint8, device=dev)
        off_np = (np.arange(n_slots + 1, dtype=np.int64) * cap)
    elif args.op == "search":
        # PIO-capture shape (phy/rmii.md:265-271): every capture is a frame whose
        # LE FCS covers its first flen - 4 bytes, so CRC32Search scans it whole
        # and finds flen - 4 (ethernet/crc.go:28-47)
        if flen is None:
            raise SystemExit("--op search needs fixed-size captures")
        fr = d_bytes[: n_local * flen].view(n_local, flen)
        starts = torch.arange(n_local, dtype=torch.int64, device=dev) * flen
        lens = torch.full((n_local,), flen - 4, dtype=torch.int32, device=dev)
        fcs = L.crc32_segments(d_bytes, starts, lens)
        fr[:, flen - 4:] = fcs.view(torch.uint8).view(n_local, 4)
        d_hit = torch.empty(n_local, dtype=torch.int64, device=dev)
    elif args.op in ("ingress", "tx_checksum", "rx_verify", "pcap") and flen is None:
        # the Zipf mix (64-1500 B on the wire) packed back to back: every frame a
        # valid UDP/IPv4 packet (rx_verify: with its LE FCS), so each takes the
        # full header-sum + UDP-sum path and is accepted
        d_lens = d_off[1:] - d_off[:-1]
        _udp4_device(L, torch, d_bytes, d_off[:-1].contiguous(), d_lens, fcs=args.op == "rx_verify")
        d_ok = torch.empty(n_local, dtype=torch.uint8, device=dev)
        d_verdict = torch.empty(n_local, dtype=torch.uint8, device=dev)
        if args.op == "tx_checksum":
            d_seg = d_off[:-1].contiguous()
            d_len = d_lens.to(torch.int32)
    elif args.op in ("ingress", "tx_checksum", "rx_verify", "pcap"):
        if flen < 42:
            raise SystemExit(f"--op {args.op} needs frames of at least 42 bytes")
        fr = d_bytes[: n_local * flen].view(n_local, flen)
        hdr = bytes.fromhex("c0ffee00dead4e8b3af9fb6b0800") + bytes([0x45, 0]) + (flen - 14).to_bytes(2, "big") \
            + bytes.fromhex("12344000401100 00c0a80a01c0a80a02".replace(" ", "")) \
            + bytes.fromhex("14e90035") + (flen - 34).to_bytes(2, "big")
        fr[:, : len(hdr)] = torch.tensor(list(hdr), dtype=torch.uint8, device=dev)
        d_ok = torch.empty(n_local, dtype=torch.uint8, device=dev)
        d_verdict = torch.empty(n_local, dtype=torch.uint8, device=dev)
        if args.op == "tx_checksum":
            # TX: the same frames as segments (start, len); the step writes the IPv4
            # header CRC and the UDP CRC in place, idempotently, every step
            d_seg = d_off[:-1].contiguous()
            d_len = (d_off[1:] - d_off[:-1]).to(torch.int32)
    sync()
    host_frames = None
    if cpu_ranks:
        hb = d_bytes.numpy().tobytes()
        host_frames = [hb[int(off_np[i]):int(off_np[i + 1])] for i in range(n_local)]

    def step():
        if cpu_ranks:
            d_crc.copy_(torch.tensor([L.crc32(f) for f in host_frames], dtype=torch.int64).to(torch.int32))
        elif args.op == "sum16":
            L.sum16_batch(d_bytes, d_seg, d_len, d_seed, out=d_sum, stream=stream)
        elif args.op == "fcs_verify":
            L.fcs_verify_batch(d_bytes, d_off, out=d_ok, stream=stream, short_frames=args.short_frames)
        elif args.op == "ingress":
            L.ingress_verify_batch(d_bytes, d_off, out=d_ok, stream=stream)
        elif args.op == "rx_verify":
            L.rx_verify_batch(d_bytes, d_off, out=(d_ok, d_verdict), stream=stream)
        elif args.op == "pcap":
            L.pcap_verify_batch(d_bytes, d_off, out=d_ok, stream=stream)
        elif args.op == "tx_checksum":
            L.tx_checksum_batch(d_bytes, d_seg, d_len, status=d_ok, stream=stream)
        elif args.op == "search":
            L.crc32_search_batch(d_bytes, d_off, out=d_hit, stream=stream)
        elif args.op == "fcs_append":
            with torch.cuda.stream(stream):
                d_len.copy_(d_len0, non_blocking=True)
            L.fcs_append_batch(d_bytes, d_start, d_len, 1536, status=d_status, stream=stream)
        elif args.op == "tx_finish":
            with torch.cuda.stream(stream):
                d_len.copy_(d_len0, non_blocking=True)
            L.tx_finish_batch(d_bytes, d_start, d_len, 1536, flags=3, status=d_status, stream=stream)
        else:
            L.crc32_batch(d_bytes, d_off, out=d_crc, stream=stream, short_frames=args.short_frames)

    # The first few hundred microseconds of launches on an idle GPU run at
    # ramping clocks (tools/prof/variants.py measured ~5 % slower kernels):
    # keep the device busy for --prewarm-s before the W warmup steps.
    t_pw = time.perf_counter()
    while time.perf_counter() - t_pw < args.prewarm_s:
        for _ in range(10):
            step()
        sync()
    for _ in range(args.warmup):
        step()
    sync()
    if dist:
        dist.barrier()
    sync()

    # The roofline's launch time: one HIP-event window on the launch stream
    # around all K timed steps (no event between steps, so the launches run
    # back to back as in the untimed ones), divided by K.  It covers every
    # launch of the entry (the plain CRC entry is the rows and the staged
    # kernel, the one that owns no slice exiting at once: DESIGN.md §3.10).
    if cpu_ranks:  # host clock around the window (no HIP events without a GPU)
        class _Ev:
            def record(self, _s):
                self.t = time.perf_counter()

            def elapsed_time(self, e):
                return (e.t - self.t) * 1e3
        ev0, ev1 = _Ev(), _Ev()
    else:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(args.steps):
        step()
    ev1.record(stream)
    sync()
    if dist:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    # the window sits inside the host clock's (both bracket the same launches)
    assert cpu_ranks or kern_ms <= 1.01 * elapsed * 1e3 / args.steps, (kern_ms, elapsed * 1e3 / args.steps)

    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=cdev)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed_max, kern_ms_max = float(t[0]), float(t[1])
    total_bytes = nbytes * world  # every rank owns the same byte count (fixed-size frames)
    if dist and flen is None:
        tb = torch.tensor([nbytes], dtype=torch.float64, device=cdev)
        dist.all_reduce(tb)
        total_bytes = int(tb.item())

    value = total_bytes * args.steps / elapsed_max / 2**30
    achieved = nbytes / (kern_ms * 1e-3) / 1e9  # GB/s, this rank's launches, HIP-event timed

    metric = {
        "crc32": "GiB/s CRC-32 over device-resident 1500B frames; % of HBM3E read peak",
        "fcs_verify": "GiB/s FCS verify (CRC-32 residue) over device-resident frames; % of HBM3E read peak",
        "sum16": "GiB/s RFC 791 internet checksum over device-resident segments; % of HBM3E read peak",
        "ingress": "GiB/s receive-path checksum verdicts (IPv4 header + UDP) over device-resident frames",
        "rx_verify": "GiB/s receive check in one pass (FCS residue + IPv4 header / UDP verdicts) over device-resident frames",
        "search": "GiB/s CRC32Search over device-resident captures (bytes scanned to the FCS hit)",
        "fcs_append": "GiB/s TX FCS append (pad, CRC-32, LE32 store) over device-resident ring slots",
        "tx_finish": "GiB/s transmit tail in one read (checksum generate + pad + FCS) over device-resident ring slots",
        "tx_checksum": "GiB/s TX checksum generate (IPv4 header + UDP) over device-resident frames",
        "pcap": "GiB/s pcap checksum re-verification (IPv4 header + UDP, capture.go semantics) over device-resident frames",
    }[args.op]
    out = {
        "metric": metric,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "prewarm_s": args.prewarm_s,
        "ms_per_step": round(elapsed_max * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 counter-hash bytes, generated on device)",
        "config": {
            "workload": desc,
            "name": wname,
            "frames_per_gpu": n_local,
            "frame_bytes": flen if flen else "zipf 64-1500",
            "bytes_per_gpu": nbytes,
            "parallelism": f"per-GPU frame partition x{world} (no collective)",
            "kernel": L.version(),
            "build_id": L.build_id(),
        },
        "pct_hbm_peak": round(100.0 * (nbytes / (elapsed_max / args.steps) / 1e9) / HBM_PEAK_GBS, 2),
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "kernel": ({"crc32": "lnx::crc32_stage_kernel<kCrc>",
                        "fcs_verify": "lnx::crc32_stage_kernel<kVerify>"} if args.short_frames else {}).get(
                args.op) or {"crc32": "lnx::crc32_rows_kernel<kCrc> + lnx::crc32_stage_kernel<kCrc> (one entry; "
                                      "each slice folded by the kernel slice_kind gives it, DESIGN.md §3.10)",
                             "fcs_verify": "lnx::crc32_rows_kernel<kVerify> + lnx::crc32_stage_kernel<kVerify>",
                       "sum16": "lnx::sum16_lines_kernel<true>",
                       "ingress": "lnx::ingress_verify_kernel + lnx::rx_verify_kernel<false, false> (one entry; "
                                  "the second works when the mean frame is under 1280 B, DESIGN.md §3.12)",
                       "rx_verify": "lnx::rx_verify_kernel<true, false>",
                       "search": "lnx::crc32_search_o_kernel",
                       "fcs_append": "lnx::crc32_rows_kernel<kAppend> (segment mode, one launch)",
                       "tx_finish": "lnx::tx_finish_kernel<FCS, CK, HBM>",
                       "tx_checksum": "lnx::ingress_verify_kernel<GEN>",
                       "pcap": "lnx::pcap_verify_kernel"}[args.op],
            "kernel_ms": round(kern_ms, 4),
            "kernel_ms_window": f"HIP events around all {args.steps} timed steps on the launch stream, / {args.steps}",
            "algorithmic_bytes_per_launch": nbytes,
        },
    }
    tag = (wname if args.op == "crc32" else f"{wname}_{args.op}") + ("_short" if args.short_frames else "")
    if args.short_frames:
        out["config"]["entry"] = "lnx_crc32_batch_ex / lnx_fcs_verify_batch_ex with LNX_BATCH_SHORT_FRAMES"
    traffic_file = os.path.join(ROOT, "profiles", f"traffic_{tag}.json")
    if os.path.exists(traffic_file):
        with open(traffic_file) as fh:
            tr = json.load(fh)
        out["roofline"]["traffic"] = tr.get("hbm_bytes_per_launch")
        out["roofline"]["traffic_source"] = os.path.relpath(traffic_file, ROOT)
    # Compute ceilings of the issue pipes (MI355X_MICROARCH.md: a wave issues a
    # VALU instruction over 2 cycles, so 0.5 wave-instructions per cycle per
    # SIMD; a ds_read_b32 wave-instruction takes 2 LDS-array cycles, so 0.5 per
    # cycle per CU; 256 CUs at 2.4 GHz), against the instruction counts per
    # launch of the committed PMC pass (profiles/counters_<tag>.json) over this
    # run's kernel time.  For kernels bound by dependent LDS / VALU chains
    # (CRC32Search) these, not HBM, say how far the kernel is from its ceiling.
    counters_file = os.path.join(ROOT, "profiles", f"counters_{tag}.json")
    if os.path.exists(counters_file) and not cpu_ranks:
        with open(counters_file) as fh:
            cn = json.load(fh)
        # the clock the profiled run held (GRBM_GUI_ACTIVE over its kernel time), else the nominal 2.4 GHz
        clk, cus = float(cn.get("clock_ghz_est") or 2.4) * 1e9, 256
        sec = kern_ms * 1e-3
        valu = cn["SQ_INSTS_VALU"] / sec
        comp = {"valu": {"achieved": round(valu / 1e9, 2), "peak": round(cus * 4 * 0.5 * clk / 1e9, 2),
                         "unit": "G wave-instr/s", "frac": round(valu / (cus * 4 * 0.5 * clk), 4),
                         "per_launch": cn["SQ_INSTS_VALU"]}}
        # LDS: the array's busy cycles (SQ_LDS_IDX_ACTIVE, bank-conflict cycles included) against one
        # array cycle per clock per CU; the instruction count beside it
        busy = cn["SQ_LDS_IDX_ACTIVE"] / sec
        comp["lds"] = {"achieved": round(busy / 1e9, 2), "peak": round(cus * clk / 1e9, 2), "unit": "G LDS-array cycles/s",
                       "frac": round(busy / (cus * clk), 4), "instr_per_launch": cn["SQ_INSTS_LDS"],
                       "bank_conflict_cycles_per_launch": cn.get("SQ_LDS_BANK_CONFLICT")}
        comp["source"] = os.path.relpath(counters_file, ROOT)
        comp["clock_ghz"] = round(clk / 1e9, 3)
        # counts from another build of the kernel say nothing about this one:
        # they are reported beside the HBM roofline, marked, and never replace it
        # (the build is the code objects' hash, lneto_amd.build_id)
        comp["same_build"] = cn.get("build_id") == L.build_id()
        out["roofline_compute"] = comp
        top = max(("valu", "lds"), key=lambda k: comp[k]["frac"])
        if comp["same_build"] and comp[top]["frac"] > out["roofline"]["frac"]:
            # the issue pipe, not HBM, is the nearer ceiling: it becomes the roofline, HBM moves beside it
            r = out["roofline"]
            r["hbm"] = {"achieved": r["achieved"], "peak": r["peak"], "unit": r["unit"], "frac": r["frac"]}
            r.update(bound=top, achieved=comp[top]["achieved"], peak=comp[top]["peak"], unit=comp[top]["unit"],
                     frac=comp[top]["frac"])

    if args.verify:
        from oracle import oracle as O
        idx = np.random.default_rng(rank).choice(n_local, min(256, n_local), replace=False)
        if args.op == "sum16":
            got = d_sum.cpu().numpy().view(np.uint16)
            seeds = d_seed.cpu().numpy().view(np.uint32)
        elif args.op in ("fcs_verify", "ingress", "tx_checksum", "pcap"):
            got = d_ok.cpu().numpy()
        elif args.op == "rx_verify":
            got = d_ok.cpu().numpy().astype(np.uint32) * 256 + d_verdict.cpu().numpy()
        elif args.op == "search":
            got = d_hit.cpu().numpy()
        elif args.op in ("fcs_append", "tx_finish"):
            got = d_status.cpu().numpy()
            lens_after = d_len.cpu().numpy()
        else:
            got = d_crc.cpu().numpy().view(np.uint32)
        for i in idx:
            s, e = int(off_np[i]), int(off_np[i + 1])
            if args.op in ("fcs_append", "tx_finish"):
                fl = int(lens[i]) if zipf_slots else flen
                s = i * 1536 if zipf_slots else s
                fr = d_bytes[s:s + fl].cpu().numpy().tobytes()
                assert int(got[i]) == 0 and int(lens_after[i]) == fl, f"frame {i}: status / length"
                assert O.crc32(fr[:-4]) == int.from_bytes(fr[-4:], "little"), f"mismatch frame {i}"
                if args.op == "tx_finish":  # the finished frame is a fixed point of both steps and is accepted
                    regen, st = O.tx_checksum(fr[:-4])
                    assert st == 0 and regen == fr[:-4] and O.ingress_verdict(fr[:-4]) == 0, f"frame {i}"
                continue
            fr = d_bytes[s:e].cpu().numpy().tobytes()
            if args.op == "sum16":
                want = O.payload_sum16(int(seeds[i]), fr)
            elif args.op == "fcs_verify":
                want = int(len(fr) >= 4 and O.crc32(fr) == 0x2144DF1C)
            elif args.op == "ingress":
                want = O.ingress_verdict(fr)
            elif args.op == "pcap":
                want = O.pcap_checksums(fr)
            elif args.op == "rx_verify":
                want = int(len(fr) >= 4 and O.crc32(fr) == 0x2144DF1C) * 256 + O.ingress_verdict(fr[:-4] if len(fr) >= 4 else b"")
            elif args.op == "tx_checksum":
                # the finished frame is a fixed point of the step and passes the receive path
                regen, st = O.tx_checksum(fr)
                assert st == 0 and regen == fr and O.ingress_verdict(fr) == 0, f"frame {i}"
                want = 0
            elif args.op == "search":
                want = O.crc32_search(fr, 0)
            else:
                want = O.crc32(fr)
            assert int(got[i]) == want, f"mismatch frame {i}"
        out["verified_sample"] = len(idx)

    if world == 1 and args.op == "crc32" and wname == "mtu1500" and not cpu_ranks and not args.no_slice16m:
        out["slice16m"] = slice16m_bench(L, synth, torch, dev)

    if args.with_copies and rank == 0:
        host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        host.copy_(d_bytes)
        hcrc = torch.empty(n_local, dtype=torch.int32, pin_memory=True)
        d2 = torch.empty_like(d_bytes)
        torch.cuda.synchronize(dev)
        reps = 5
        t1 = time.perf_counter()
        for _ in range(reps):
            d2.copy_(host, non_blocking=True)
            L.crc32_batch(d2, d_off, out=d_crc, stream=stream)
            hcrc.copy_(d_crc, non_blocking=True)
        torch.cuda.synchronize(dev)
        el = (time.perf_counter() - t1) / reps
        out["pcie_inclusive"] = {"value": round(nbytes / el / 2**30, 2), "unit": "GiB/s",
                                 "note": "pinned H2D of frames + kernel + D2H of CRCs, serial, 1 stream"}

    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.op not in ("fcs_append", "tx_checksum",
                                                                                  "tx_finish"):
        out["cpu_baseline"] = cpu_baseline(d_bytes, off_np, flen, budget_s=args.cpu_budget, op=args.op)

    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
