#!/usr/bin/env python3
"""bench.py -- round-trip DEFLATE+INFLATE throughput of libdmx on MI355X.

Metric (BASELINE.json): "GB/s deflate+inflate on 1 GiB buffer at 1/2/4/8 MI355X; ratio vs
reference".  One step = deflate of a 1 GiB device-resident shard per GPU (level 2, the
reference's "fast" level, configs[1]: 1 GiB zero/repeat synthetic buffer) followed by
inflate of the produced stream back into HBM.  With N > 1 GPUs a step is the
distributed round trip of ONE stream: every rank compresses its shard in sub-shards whose
bytes travel to rank 0 over RCCL while the next sub-shard compresses (the north_star's "final
bitstream gather", shard.deflate_gather); rank 0 indexes the gathered stream's segment starts,
proves the cut candidates (dmx_segment_check_device) and scatters one piece per rank; every
rank inflates its piece (pieces after the first in piece mode), and the decoded bytes stay
where they were decoded (shard.scatter_inflate, gather=False).  value = total uncompressed
bytes of all ranks / max-over-ranks step time.

  python bench.py                          # N=1, defaults (+ the per-config sub-records)
  torchrun --nproc-per-node N bench.py --gpus N [--strong]

Prints ONE JSON line on rank 0.  Besides the contract fields it carries, at N = 1:
  corpora      the same round trip on the other Appendix-B corpora (1 GiB each): GB/s per
               direction, ratio next to the reference's level-2 ratio and zlib-1's, the
               roofline fraction of each direction's kernels
  c3_inflate   config C3: inflate of the zlib level-1 stream of the 25,165,962-B large.bmp
               stand-in (block-parallel path for marker-less streams) and of libdmx's own
               stream of it, bit-exact checked
  c5_level3    config C5: level 3 on the 1 GiB text corpus, ratio next to the reference L3's
               and zlib-6's
  c4_64k       config C4's 64 KiB blocks: the mixed round trip with segment_bytes = 65536
  cpu_baseline the reference compiled from its headers (oracle/_ref), 1 core and `nproc`
               processes on disjoint slices, with the host CPU model
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))

import dmx  # noqa: E402
import shard  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
GiB = 1 << 30
C3_N = 25165962  # large.bmp stand-in
# reference ratios measured in the survey container
REF_RATIO_L2 = {"zeros": 96.0938, "repeat": 19.6319, "text": 2.0892, "random": 0.9998,
                "mixed": 2.4723, "bmp": 3.315}
REF_NOTES = {"text": "reference L2 stream is lossy (SURVEY A-1)",
             "mixed": "reference L2 stream is invalid (SURVEY A-3)",
             "bmp": "reference L2 stream is invalid (SURVEY A-3)"}
REF_RATIO_L3_TEXT = 2.5741  # reference L3 on the 1 MiB text prefix
PROFILE_TAG = "r06"  # tools/profile_all.sh writes profiles/<tag>_kstats_*.csv and traffic.json


def profile_path(name):
    """profiles/<tag>_<name> of THIS round's kernels, or None: an earlier round's profile
    describes other kernels and is never cited."""
    rel = f"profiles/{PROFILE_TAG}_{name}"
    return rel if os.path.exists(os.path.join(ROOT, rel)) else None
TRAFFIC_JSON = os.path.join(ROOT, "profiles", "traffic.json")


def traffic_entry(tj, key):
    """HBM bytes per launch under key, only when measured this round (traffic.py records the
    round tag with every entry); None otherwise."""
    d = tj.get(key + ":detail")
    if key not in tj or not isinstance(d, dict) or d.get("round") != PROFILE_TAG:
        return None
    return tj[key]


def traffic_of(key_prefix, kernels):
    """HBM bytes per launch from profiles/traffic.json (tools/profile_all.sh) for each kernel
    that has an entry of this round under key_prefix + kernel; None when none has."""
    try:
        tj = json.load(open(TRAFFIC_JSON))
    except Exception:
        return None
    got = {k: traffic_entry(tj, key_prefix + k) for k in kernels}
    got = {k: v for k, v in got.items() if v is not None}
    return got or None


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--corpus", default="repeat", choices=sorted(dmx.CORPUS))
    p.add_argument("--bytes", type=int, default=GiB,
                   help="uncompressed bytes per GPU (weak scaling) or in total (--strong)")
    p.add_argument("--strong", action="store_true", help="fixed total size split over the ranks")
    p.add_argument("--level", type=int, default=2)
    p.add_argument("--segment", type=int, default=32768)
    p.add_argument("--cpu-sample", type=int, default=64 << 20,
                   help="bytes of the same corpus the single-core reference baseline compresses")
    p.add_argument("--cpu-slice", type=int, default=16 << 20,
                   help="bytes per process of the nproc-process reference baseline")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extras", action="store_true", help="skip the per-config sub-records")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    p.add_argument("--sub", type=int, default=4, help="N > 1: sub-shards per rank in the pipelined gather")
    return p.parse_args()


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(kind, nbytes, level, slice_bytes):
    """Reference deflate::compress + inflate::decompress on the host cores (oracle/_ref):
    (a) one thread on `nbytes`; (b) P processes on disjoint `slice_bytes` slices, started
    together, wall-clock aggregate (SURVEY 8(d) "Timing method (CPU reference)")."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_bind import Reference
    if not Reference.available():
        return {"error": "oracle/_ref/libdeflate_ref.so absent (built only where /root/reference exists)"}
    data = dmx.corpus(kind, nbytes)
    ref = Reference()
    t0 = time.perf_counter()
    comp = ref.compress(data, level)
    t1 = time.perf_counter()
    try:
        ref.decompress(comp)
        t2 = time.perf_counter()
    except Exception:
        t2 = t1 + float("nan")
    secs = t2 - t0
    res = {"value": round(nbytes / secs / 1e9, 6), "unit": "GB/s", "cores": 1, "kind": "reference",
           "sample": f"{nbytes >> 20} MiB of the {kind} corpus, reference deflate::compress level {level} "
                     f"+ inflate::decompress (oracle/_ref, g++ -O2), single thread",
           "deflate_GBps": round(nbytes / (t1 - t0) / 1e9, 6),
           "inflate_GBps": round(nbytes / (t2 - t1) / 1e9, 6),
           "ratio": round(nbytes / len(comp), 4), "cpu_model": cpu_model()}
    # (b) P processes on disjoint slices; the box's CPU share is 16 per GPU
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    P = max(1, min(16, ncpu))
    worker = os.path.join(ROOT, "tests", "cpu_ref_worker.py")
    procs = [subprocess.Popen([sys.executable, worker, kind, str(i * slice_bytes), str(slice_bytes), str(level)],
                              stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True) for i in range(P)]
    for pr in procs:
        if pr.stdout.readline().strip() != "ready":
            raise RuntimeError("cpu worker failed to start")
    w0 = time.perf_counter()
    for pr in procs:
        pr.stdin.write("go\n")
        pr.stdin.flush()
    outs = [json.loads(pr.stdout.readline()) for pr in procs]
    wall = time.perf_counter() - w0
    for pr in procs:
        pr.wait(timeout=60)
    tot = P * slice_bytes
    res["nproc"] = {"value": round(tot / wall / 1e9, 6), "unit": "GB/s", "cores": P,
                    "sample": f"{P} processes x {slice_bytes >> 20} MiB disjoint slices of the {kind} corpus, "
                              f"deflate level {level} + inflate each, wall clock from a common start",
                    "deflate_s_max": round(max(o["deflate_s"] for o in outs), 3),
                    "inflate_s_max": round(max(o["inflate_s"] for o in outs), 3)}
    return res


class Runner:
    """Device-resident deflate + inflate of one shard on one GPU (buffers reused across corpora)."""

    def __init__(self, torch, ctx, dev, n, stream):
        self.torch, self.ctx, self.dev, self.n, self.stream = torch, ctx, dev, n, stream
        self.bound = dmx.deflate_bound(n) + 64
        self.d_in = torch.empty(n + 64, dtype=torch.uint8, device=dev)
        self.d_comp = torch.empty(self.bound, dtype=torch.uint8, device=dev)
        self.out_cap = n + 64
        self.d_out = torch.empty(self.out_cap, dtype=torch.uint8, device=dev)

    def grow_out(self, cap):
        """N > 1: a rank decodes a piece of the whole stream, whose size follows the cuts."""
        self.out_cap = cap
        self.d_out = self.torch.empty(cap, dtype=self.torch.uint8, device=self.dev)

    def load(self, kind, offset):
        torch = self.torch
        host = torch.empty(self.n, dtype=torch.uint8).pin_memory()
        dmx.corpus_into(kind, self.n, host.data_ptr(), offset=offset)
        self.d_in[: self.n].copy_(host)
        del host

    def step(self, level, not_final=False, gather=None):
        """One round trip; returns (events, clen, olen, deflate stats, inflate stats)."""
        torch, n, sh = self.torch, self.n, self.stream.cuda_stream
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record(self.stream)
        clen = self.ctx.deflate_device(self.d_in.data_ptr(), n, level, self.d_comp.data_ptr(), self.bound,
                                       stream=sh, not_final=not_final)
        ks_d = self.ctx.stats()
        ev[1].record(self.stream)
        if gather is not None:
            gather(self.d_comp, clen)
        ev[2].record(self.stream)
        ilen = clen
        if not_final:  # make the shard a complete stream for the local round trip
            self.d_comp[clen: clen + 2].copy_(torch.tensor([0x03, 0x00], dtype=torch.uint8, device=self.dev))
            ilen = clen + 2
        olen = self.ctx.inflate_device(self.d_comp.data_ptr(), ilen, self.d_out.data_ptr(), n + 64, stream=sh)
        ks_i = self.ctx.stats()
        ev[3].record(self.stream)
        return ev, clen, olen, ks_d, ks_i

    def verify(self, olen):
        return olen == self.n and bool(self.torch.equal(self.d_out[: self.n], self.d_in[: self.n]))


class _NoEvent:
    """Stand-in for torch.cuda.Event on a CPU device (the gloo tests of dist_step)."""

    def record(self, *a):
        pass

    def elapsed_time(self, other):
        return 0.0


def dist_step(torch, ctx, dev, run, level, gathered, sub, stream):
    """One distributed round trip (N > 1, see the module doc); returns (events, stream bytes,
    this rank's decoded bytes, ok of the split)."""
    import torch.distributed as dist
    rank = dist.get_rank()
    ev = [torch.cuda.Event(enable_timing=True) if dev.type == "cuda" else _NoEvent() for _ in range(3)]
    ev[0].record(stream)
    total, _ = shard.deflate_gather(ctx, run.d_in, run.n, level, out=gathered, sub=sub)
    ev[1].record(stream)
    # the packed stream and the pieces are written by torch copies: the codec runs on torch's
    # stream so it reads them after those copies
    sh = torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else None
    starts, check = None, None
    if rank == 0:
        starts = ctx.segment_starts_device(gathered.data_ptr(), total, stream=sh)
        check = lambda c: ctx.segment_check_device(gathered.data_ptr(), total, c, stream=sh)  # noqa: E731
    got = [0]

    def decode(piece, first):
        fn = ctx.inflate_device if first else ctx.inflate_piece_device
        olen = fn(piece.data_ptr(), piece.numel(), run.d_out.data_ptr(), run.out_cap, stream=sh)
        got[0] = olen
        return run.d_out[:olen]

    # the pieces decode with no host sync (dmx_inflate_device_async): their {bytes, status} words
    # ride in the ranks' one all_gather; a piece the lane path does not take decodes again
    # synchronously (decode above)
    d_res = torch.zeros(2, dtype=torch.int64, device=dev)

    def decode_async(piece, first):
        ctx.inflate_device_async(piece.data_ptr(), piece.numel(), run.d_out.data_ptr(), run.out_cap,
                                 d_res.data_ptr(), stream=sh, piece=not first)
        return d_res, run.d_out

    src = gathered if rank == 0 else torch.empty(0, dtype=torch.uint8, device=dev)
    _, ok = shard.scatter_inflate(src, total if rank == 0 else 0, decode, starts=starts,
                                  out=run.d_out if rank == 0 else None, check=check, gather=False,
                                  balance="count", decode_async=decode_async if hasattr(ctx, "inflate_device_async") else None)
    ev[2].record(stream)
    if not got[0]:  # decoded by decode_async: this rank's bytes
        got[0] = int(d_res[0].item()) if int(d_res[1].item()) == 0 else got[0]
    return ev, total, got[0], ok


def dist_verify(torch, dist, run, corpus, olen, ok, dev, total_n):
    """Each rank's decoded piece against the corpus bytes at its output offset (outside the
    timed region); a fallen-back split is checked whole on rank 0."""
    rank = dist.get_rank()
    # a fallen-back split decoded the whole stream on rank 0 (the other ranks' pieces are moot)
    sizes = shard.gather_sizes(olen if (ok or rank == 0) else 0, dev)
    off = sum(sizes[:rank])
    good = True
    m = sizes[rank]
    if sum(sizes) != total_n:
        good = False
    step = 256 << 20
    host = torch.empty(min(step, max(m, 1)), dtype=torch.uint8)
    if dev.type == "cuda":
        host = host.pin_memory()
    for b in range(0, m, step):
        k = min(step, m - b)
        dmx.corpus_into(corpus, k, host.data_ptr(), offset=off + b)
        if not torch.equal(run.d_out[b:b + k], host[:k].to(dev)):
            good = False
            break
    t = torch.tensor([1 if good else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def summarize(recs, n):
    t_def = sum(r[0][0].elapsed_time(r[0][1]) for r in recs) / len(recs)
    t_gat = sum(r[0][1].elapsed_time(r[0][2]) for r in recs) / len(recs)
    t_inf = sum(r[0][2].elapsed_time(r[0][3]) for r in recs) / len(recs)
    k_def = sum(r[3].ms_main_kernel for r in recs) / len(recs)
    k_inf = sum(r[4].ms_main_kernel for r in recs) / len(recs)
    clen = recs[-1][1]
    alg = n + clen
    return {"t_def": t_def, "t_gat": t_gat, "t_inf": t_inf, "k_def": k_def, "k_inf": k_inf,
            "clen": clen, "alg": alg, "path": int(recs[-1][4].path),
            "frac_def": alg / (k_def * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            "frac_inf": alg / (k_inf * 1e-3) / 1e9 / HBM_PEAK_GBPS}


DEF_KERNELS = ["k_deflate_segments", "k_deflate_emit"]  # front (match + parse), entropy + bit packing
DEF_KERNEL = "+".join(DEF_KERNELS)
INF_KERNEL = {3: "k_inflate_pj", 4: "k_inflate_lanes+k_inflate_resolve",
              5: "k_fb_decode+k_fb_resolve (block-parallel)", 2: "k_inflate_serial"}


def zlib_ratio(kind, level, nbytes=16 << 20, chunk=None):
    """zlib's ratio on a 16 MiB sample: one stream, or (chunk) independent chunks -- the
    constraint libdmx's segments and the reference's 32 KiB chunks work under."""
    d = dmx.corpus(kind, nbytes)
    step = chunk or len(d)
    tot = 0
    for i in range(0, len(d), step):
        z = zlib.compressobj(level, zlib.DEFLATED, -15)
        tot += len(z.compress(d[i:i + step]) + z.flush())
    return round(len(d) / tot, 4)


def corpus_record(run, kind, level, steps, tag=None):
    """tag: the key of this record's profiles and PMC traffic (default: the corpus)."""
    tag = tag or kind
    run.load(kind, 0)
    run.step(level)
    ev, clen, olen, _, _ = run.step(level)
    ok = run.verify(olen)
    recs = [run.step(level) for _ in range(steps)]
    run.torch.cuda.synchronize(run.dev)
    s = summarize(recs, run.n)
    n = run.n
    inf_k = ["k_inflate_lanes", "k_inflate_resolve", "k_inflate_resolve_wave", "k_inflate_resolve_half",
             "k_inflate_resolve_half_wave", "k_inflate_pj_list"]
    return {"bytes": n, "level": level, "roundtrip_ok": ok,
            "roundtrip_GBps": round(n / ((s["t_def"] + s["t_inf"]) * 1e-3) / 1e9, 3),
            "deflate_GBps": round(n / (s["t_def"] * 1e-3) / 1e9, 3),
            "inflate_GBps": round(n / (s["t_inf"] * 1e-3) / 1e9, 3),
            "ratio": round(n / s["clen"], 4),
            "ref_ratio_L2": REF_RATIO_L2.get(kind), "ref_note": REF_NOTES.get(kind, "reference L2 round-trips"),
            "zlib1_ratio_16MiB": zlib_ratio(kind, 1),
            "zlib1_ratio_32KiB_chunks_16MiB": zlib_ratio(kind, 1, chunk=32768),
            "kernel_ms": {DEF_KERNEL: round(s["k_def"], 4),
                          INF_KERNEL.get(s["path"], "k_inflate_segments"): round(s["k_inf"], 4)},
            "inflate_path": s["path"],
            "alg_bytes": s["alg"],
            "roofline_frac": {"deflate": round(s["frac_def"], 5), "inflate": round(s["frac_inf"], 5)},
            "traffic": {"deflate": traffic_of(f"{tag}:{n}:{level}:", DEF_KERNELS),
                        "inflate": traffic_of(f"{tag}:{n}:{level}:", inf_k)},
            "profile": profile_path(f"kstats_{tag}_L{level}.csv")}


def c4_record(run, dev, level, steps):
    """Config C4's block size: the mixed corpus as 64 KiB DEFLATE blocks (one
    Huffman block per 64 KiB of input, its two 32 KiB halves matched independently), the same
    round trip as the corpora records (whose mixed entry is at 32 KiB segments), on this GPU's
    1 GiB shard; the 8-GPU gather of C4 is the N > 1 bench step."""
    ctx64 = dmx.Context(device=dev.index or 0, segment_bytes=65536)
    ctx64.set_timing(True)
    saved = run.ctx
    run.ctx = ctx64
    try:
        rec = corpus_record(run, "mixed", level, steps, tag="c4_64k")
    finally:
        run.ctx = saved
        ctx64.close()
    rec["segment_bytes"] = 65536
    return rec


def c3_record(torch, ctx, dev, stream):
    """Config C3: inflate of large.bmp's zlib-1 raw stream and of libdmx's
    own level-2 stream of it (C3 (ii)); output bit-exact to the original (= the reference's
    inflate output, tests/golden/manifest.json c3_bmp_zlib1)."""
    data = dmx.corpus("bmp", C3_N)
    z = zlib.compressobj(1, zlib.DEFLATED, -15)
    s = z.compress(data) + z.flush()
    ref = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    out = torch.empty(C3_N + 64, dtype=torch.uint8, device=dev)
    res = {"n": C3_N, "sha256_out_expected": hashlib.sha256(data).hexdigest()[:16]}
    streams = {"zlib1": s, "libdmx_L2": ctx.compress(data, 2)}
    for name, st in streams.items():
        d_s = torch.frombuffer(bytearray(st), dtype=torch.uint8).to(dev)
        ms = []
        for it in range(8):
            olen = ctx.inflate_device(d_s.data_ptr(), len(st), out.data_ptr(), C3_N + 64,
                                      stream=stream.cuda_stream)
            if it >= 3:
                ms.append(ctx.stats().ms_device_total)
        ms.sort()
        med = ms[len(ms) // 2]
        ok = olen == C3_N and bool(torch.equal(out[:C3_N], ref))
        res[name] = {"stream_bytes": len(st), "inflate_ms": round(med, 3),
                     "inflate_GBps": round(C3_N / (med * 1e-3) / 1e9, 3), "path": int(ctx.stats().path),
                     "roofline_frac": round((C3_N + len(st)) / (med * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5),
                     "bit_exact": ok}
    res["zlib1"]["traffic"] = traffic_of("c3_zlib1:", ["k_fb_scan", "k_fb_compact", "k_fb_check", "k_fb_pdecode", "k_fb_units",
                                                       "k_fb_win_init", "k_fb_win_jump", "k_fb_final"])
    res["zlib1"]["profile"] = profile_path("kstats_c3_zlib1.csv")
    return res


FOREIGN_REF_MBPS = {"text": 35.1, "mixed": 48.2, "zeros": 227.6}  # reference inflate of zlib-1, 1 GiB


def foreign_record(torch, ctx, dev, stream, kind="text", nbytes=GiB, pieces=8):
    """A third-party stream at BASELINE scale on path 5: zlib level 1 of
    the 1 GiB corpus, compressed on `pieces` host threads (zlib releases the GIL) as one raw
    stream -- every piece primed with the previous 32 KiB as its dictionary, joined at sync
    flushes (an empty stored block each) -- so matches cross the joins as in one zlib run.  The
    output's SHA-256 is checked against SURVEY Appendix B (tests/test_gpu_foreign_1GiB.py runs
    the whole-stream zlib-1 of text, mixed and zeros)."""
    from concurrent.futures import ThreadPoolExecutor
    data = dmx.corpus(kind, nbytes)
    step = -(-nbytes // pieces)

    def comp(i):
        b = i * step
        z = zlib.compressobj(1, zlib.DEFLATED, -15, zdict=data[max(b - 32768, 0):b]) if b else \
            zlib.compressobj(1, zlib.DEFLATED, -15)
        out = z.compress(data[b:b + step])
        return out + (z.flush() if b + step >= nbytes else z.flush(zlib.Z_SYNC_FLUSH))

    with ThreadPoolExecutor(pieces) as ex:
        s = b"".join(ex.map(comp, range(pieces)))
    sha = hashlib.sha256(data).hexdigest()
    del data
    d_s = torch.frombuffer(bytearray(s), dtype=torch.uint8).to(dev)
    out = torch.empty(nbytes + 64, dtype=torch.uint8, device=dev)
    ms = []
    for it in range(4):
        olen = ctx.inflate_device(d_s.data_ptr(), len(s), out.data_ptr(), nbytes + 64, stream=stream.cuda_stream)
        if it >= 1:
            ms.append(ctx.stats().ms_device_total)
    path = int(ctx.stats().path)
    ok = olen == nbytes and hashlib.sha256(out[:nbytes].cpu().numpy().tobytes()).hexdigest() == sha
    med = sorted(ms)[len(ms) // 2]
    ref = FOREIGN_REF_MBPS.get(kind)
    return {"corpus": kind, "bytes": nbytes, "stream": f"zlib level 1, {pieces} pieces joined at sync flushes, "
                                                       "each primed with the previous 32 KiB",
            "stream_bytes": len(s), "inflate_ms": round(med, 3), "inflate_GBps": round(nbytes / (med * 1e-3) / 1e9, 3),
            "path": path, "sha256_ok": ok,
            "roofline_frac": round((nbytes + len(s)) / (med * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5),
            "ref_inflate_MBps_survey6": ref,
            "vs_reference_1core": round(nbytes / (med * 1e-3) / 1e6 / ref, 1) if ref else None}


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    ctx = dmx.Context(device=local, segment_bytes=a.segment)
    ctx.set_timing(True)
    if a.strong:  # fixed total: rank r takes its segment-aligned share
        b, e = shard.shard_range(a.bytes, rank, world, a.segment)
        n, offset = max(e - b, 0), b
    else:
        n, offset = a.bytes, rank * a.bytes
    stream = torch.cuda.current_stream(dev)
    run = Runner(torch, ctx, dev, n, stream)
    run.load(a.corpus, offset)
    last = rank == world - 1
    total_bytes = a.bytes if a.strong else world * n
    recs = []
    split_ok = True
    if world == 1:
        for _ in range(a.warmup):
            run.step(a.level)
        # correctness of the round trip (outside the timed region)
        _, clen, olen, _, _ = run.step(a.level)
        ok = run.verify(olen)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            recs.append(run.step(a.level))
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
    else:
        # the whole stream lands on rank 0; every rank's decoded piece is sized by the cuts
        gathered = torch.empty(world * run.bound + 64, dtype=torch.uint8, device=dev) if rank == 0 else None
        run.grow_out(total_bytes + 64 if rank == 0 else 2 * max(n, 1) + (64 << 20))
        for _ in range(a.warmup):
            dist_step(torch, ctx, dev, run, a.level, gathered, a.sub, stream)
        _, _, olen, split_ok = dist_step(torch, ctx, dev, run, a.level, gathered, a.sub, stream)
        torch.cuda.synchronize(dev)
        ok = dist_verify(torch, dist, run, a.corpus, olen, split_ok, dev, total_bytes)
        dist_recs = []
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            dist_recs.append(dist_step(torch, ctx, dev, run, a.level, gathered, a.sub, stream))
        torch.cuda.synchronize(dev)
        dist.barrier()
        elapsed = time.perf_counter() - t0
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        split_ok = all(r[3] for r in dist_recs)
        t_dg = sum(r[0][0].elapsed_time(r[0][1]) for r in dist_recs) / len(dist_recs)
        t_si = sum(r[0][1].elapsed_time(r[0][2]) for r in dist_recs) / len(dist_recs)
        # kernel times and the roofline: this rank's shard as one local round trip, after the
        # timed region (the distributed step launches per sub-shard and per piece)
        run.grow_out(n + 64)
        for _ in range(2):
            run.step(a.level)
        recs = [run.step(a.level) for _ in range(3)]
        torch.cuda.synchronize(dev)

    # practical HBM ceiling: a device-to-device copy of the shard, after the timed
    # region, on torch's current stream where its events are recorded; bytes = N read + N written
    copy_ms = 1e9
    for _ in range(3):
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record()
        run.d_out[:n].copy_(run.d_in[:n])
        c1.record()
        c1.synchronize()
        copy_ms = min(copy_ms, c0.elapsed_time(c1))
    d2d_gbps = 2 * n / (copy_ms * 1e-3) / 1e9

    ms_step = elapsed / a.steps * 1e3
    s = summarize(recs, n)
    ratio = n / s["clen"]
    # roofline of the dominant kernel: algorithmic bytes = N read + C written (deflate) or
    # C read + N written (inflate), per launch, over its HIP-event duration
    inf_kernel = INF_KERNEL.get(s["path"], "k_inflate_segments")
    # (deflate is two back-to-back kernels, front + emission: the HIP-event window spans both,
    # and its traffic is the sum of the two kernels' PMC bytes per launch)
    dom = inf_kernel if s["k_inf"] >= s["k_def"] else DEF_KERNEL
    kms = max(s["k_inf"], s["k_def"])
    achieved = s["alg"] / (kms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(a.traffic_json):
        try:
            tj = json.load(open(a.traffic_json))
            parts = [traffic_entry(tj, f"{a.corpus}:{n}:{a.level}:{k}") for k in dom.split("+")]
            traffic = sum(parts) if all(x is not None for x in parts) else None
        except Exception:
            traffic = None

    res = None
    if rank == 0:
        res = {
            "metric": "GB/s deflate+inflate on 1 GiB buffer at 1/2/4/8 MI355X; ratio vs reference",
            "value": round(total_bytes / (ms_step * 1e-3) / 1e9, 4),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if a.strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": f"deflate level {a.level} + inflate round trip of a "
                                   f"{'total' if a.strong else 'per-GPU'} {a.bytes / GiB:g} GiB '{a.corpus}' "
                                   f"corpus (SURVEY App. B), device-resident",
                       "corpus": a.corpus, "bytes_per_gpu": n, "level": a.level,
                       "segment_bytes": a.segment, "parallelism": f"shard{world}"},
            "roundtrip_ok": ok,
            "deflate_GBps": round(total_bytes / (s["t_def"] * 1e-3) / 1e9, 4),
            "inflate_GBps": round(total_bytes / (s["t_inf"] * 1e-3) / 1e9, 4),
            "gather_ms": round(s["t_gat"], 4),
            "ratio": round(ratio, 4),
            "ref_ratio": REF_RATIO_L2.get(a.corpus) if a.level == 2 else None,
            "ref_ratio_note": REF_NOTES.get(a.corpus, "reference L2 stream round-trips"),
            "kernel_ms": {DEF_KERNEL: round(s["k_def"], 4), inf_kernel: round(s["k_inf"], 4)},
            "inflate_path": s["path"],
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5),
                         "traffic": traffic, "kernel": dom,
                         "alg_bytes_per_launch": s["alg"],
                         "frac_deflate": round(s["frac_def"], 5), "frac_inflate": round(s["frac_inf"], 5),
                         "d2d_copy_GBps": round(d2d_gbps, 1)},
            "cpu_baseline": None,
        }
        if world > 1:
            res.update({
                "deflate_GBps": round(total_bytes / (t_dg * 1e-3) / 1e9, 4),
                "inflate_GBps": round(total_bytes / (t_si * 1e-3) / 1e9, 4),
                "gather_ms": None,
                "distributed": {"deflate_gather_ms": round(t_dg, 4), "scatter_inflate_ms": round(t_si, 4),
                                "sub_shards": a.sub, "split_ok": split_ok,
                                "note": "one stream: sub-shard deflate with the gather to rank 0 pipelined "
                                        "behind it (RCCL P2P), proven cuts, piece-mode inflate on every rank; "
                                        "decoded bytes stay on the rank that decoded them; kernel_ms / roofline "
                                        "from a local round trip of rank 0's shard after the timed region"}})
    if world == 1 and not a.no_extras:
        # sub-records (outside the timed region): the other corpora, C3 and C5
        extras = {}
        for kind in ("text", "mixed", "random", "zeros", "bmp"):
            if kind != a.corpus:
                extras[kind] = corpus_record(run, kind, a.level, 3)
        res["corpora"] = extras
        res["c5_level3"] = corpus_record(run, "text", 3, 3)
        res["c5_level3"].update({"ref_ratio_L3_1MiB": REF_RATIO_L3_TEXT, "zlib6_ratio_16MiB": zlib_ratio("text", 6),
                                 "zlib6_ratio_32KiB_chunks_16MiB": zlib_ratio("text", 6, chunk=32768)})
        res["c3_inflate"] = c3_record(torch, ctx, dev, stream)
        res["c4_64k"] = c4_record(run, dev, a.level, 3)
        res["foreign_1GiB"] = foreign_record(torch, ctx, dev, stream)
    if rank == 0:
        if world == 1 and not a.no_cpu_baseline:
            try:
                res["cpu_baseline"] = cpu_baseline(a.corpus, min(a.cpu_sample, n), a.level, a.cpu_slice)
            except Exception as e:  # the baseline is informative, never fatal
                res["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(res), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
