#!/usr/bin/env python3
"""bench.py -- round-trip DEFLATE+INFLATE throughput of libdmx on MI355X.

Metric (BASELINE.json): "GB/s deflate+inflate on 1 GiB buffer at 1/2/4/8 MI355X; ratio vs
reference".  One step = deflate of a 1 GiB device-resident shard per GPU (level 2, the
reference's "fast" level, configs[1]: 1 GiB zero/repeat synthetic buffer) followed by
inflate of the produced stream back into HBM; with N > 1 GPUs the compressed shards are also
gathered to rank 0 over RCCL (the north_star's "final bitstream gather").  value = total
uncompressed bytes of all ranks / max-over-ranks step time.

  python bench.py                          # N=1, defaults
  torchrun --nproc-per-node N bench.py --gpus N

Prints ONE JSON line on rank 0.  Extra fields: per-phase GB/s, compression ratio next to the
reference's ratio on the same corpus, the roofline of the dominant kernel (HIP-event timed
on the stream it runs on), and the reference CPU baseline timed on this host (rank 0, N=1).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))

import dmx  # noqa: E402
import shard  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
GiB = 1 << 30
# reference ratios measured in the survey container
REF_RATIO_L2 = {"zeros": 96.0938, "repeat": 19.6319, "text": 2.0892, "random": 0.9998,
                "mixed": 2.4723, "bmp": 3.315}
REF_NOTES = {"text": "reference L2 stream is lossy (SURVEY A-1)",
             "mixed": "reference L2 stream is invalid (SURVEY A-3)",
             "bmp": "reference L2 stream is invalid (SURVEY A-3)"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--corpus", default="repeat", choices=sorted(dmx.CORPUS))
    p.add_argument("--bytes", type=int, default=GiB, help="uncompressed bytes per GPU")
    p.add_argument("--level", type=int, default=2)
    p.add_argument("--segment", type=int, default=32768)
    p.add_argument("--cpu-sample", type=int, default=64 << 20,
                   help="bytes of the same corpus the reference CPU baseline compresses")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    return p.parse_args()


def cpu_baseline(kind_corpus, nbytes, level):
    """Reference deflate::compress + inflate::decompress on one host core (oracle/_ref)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_bind import Reference, Oracle
    data = dmx.corpus(kind_corpus, nbytes)
    if Reference.available():
        ref = Reference()
        t0 = time.perf_counter()
        comp = ref.compress(data, level)
        t1 = time.perf_counter()
        try:
            ref.decompress(comp)
            t2 = time.perf_counter()
        except Exception:
            t2 = t1 + float("nan")
        secs = (t1 - t0) + (t2 - t1)
        return {"value": round(nbytes / secs / 1e9, 6), "unit": "GB/s", "cores": 1, "kind": "reference",
                "sample": f"{nbytes >> 20} MiB of the {kind_corpus} corpus, reference deflate::compress "
                          f"level {level} + inflate::decompress (oracle/_ref, g++ -O2), single thread",
                "deflate_GBps": round(nbytes / (t1 - t0) / 1e9, 6),
                "inflate_GBps": round(nbytes / (t2 - t1) / 1e9, 6),
                "ratio": round(nbytes / len(comp), 4)}
    # restatement: only the inflate is restated in C (oracle/inflate_oracle.c)
    orc = Oracle()
    comp = dmx.compress(data, level)
    t0 = time.perf_counter()
    orc.inflate(comp)
    secs = time.perf_counter() - t0
    return {"value": round(nbytes / secs / 1e9, 6), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"{nbytes >> 20} MiB {kind_corpus}: oracle inflate only (oracle/_ref absent)"}


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
    n = a.bytes

    # input shard r = bytes [r*n, (r+1)*n) of the corpus, generated on the host, copied to HBM
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    dmx.corpus_into(a.corpus, n, host.data_ptr(), offset=rank * n)
    d_in = host.to(dev, non_blocking=False)
    del host
    bound = dmx.deflate_bound(n) + 64
    d_comp = torch.empty(bound, dtype=torch.uint8, device=dev)
    d_out = torch.empty(n + 64, dtype=torch.uint8, device=dev)
    last = rank == world - 1
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    tail = torch.tensor([0x03, 0x00], dtype=torch.uint8, device=dev)  # final empty fixed block
    gathered = None
    if world > 1 and rank == 0:
        gathered = torch.empty(world * bound, dtype=torch.uint8, device=dev)

    def step(record):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record(stream)
        clen = ctx.deflate_device(d_in.data_ptr(), n, a.level, d_comp.data_ptr(), bound, stream=sh,
                                  not_final=not last)
        ks_d = ctx.stats()
        ev[1].record(stream)
        if world > 1:  # RCCL gather of the compressed shards to rank 0 (xGMI P2P)
            shard.gather_stream(d_comp, clen, gathered)
        ev[2].record(stream)
        ilen = clen
        if not last:  # make the shard a complete stream for the local round trip
            d_comp[clen: clen + 2].copy_(tail)
            ilen = clen + 2
        olen = ctx.inflate_device(d_comp.data_ptr(), ilen, d_out.data_ptr(), n + 64, stream=sh)
        ks_i = ctx.stats()
        ev[3].record(stream)
        if record is not None:
            record.append((ev, clen, olen, ks_d, ks_i))
        return clen, olen

    for _ in range(a.warmup):
        step(None)
    # correctness of the round trip (outside the timed region)
    clen, olen = step(None)
    ok = olen == n and torch.equal(d_out[:n], d_in)

    recs = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(recs)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        okt = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())

    # practical HBM ceiling: a device-to-device copy of the shard, after the timed
    # region, on torch's current stream where its events are recorded; bytes = N read + N written
    copy_ms = 1e9
    for _ in range(3):
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record()
        d_out[:n].copy_(d_in)
        c1.record()
        c1.synchronize()
        copy_ms = min(copy_ms, c0.elapsed_time(c1))
    d2d_gbps = 2 * n / (copy_ms * 1e-3) / 1e9

    ms_step = elapsed / a.steps * 1e3
    t_def = sum(r[0][0].elapsed_time(r[0][1]) for r in recs) / len(recs)
    t_gat = sum(r[0][1].elapsed_time(r[0][2]) for r in recs) / len(recs)
    t_inf = sum(r[0][2].elapsed_time(r[0][3]) for r in recs) / len(recs)
    k_def = sum(r[3].ms_main_kernel for r in recs) / len(recs)
    k_inf = sum(r[4].ms_main_kernel for r in recs) / len(recs)
    comp_bytes = recs[-1][1]
    ratio = n / comp_bytes
    # roofline of the dominant kernel: algorithmic bytes = N read + C written (deflate) or
    # C read + N written (inflate), per launch, over its HIP-event duration
    alg = n + comp_bytes
    path = recs[-1][4].path
    inf_kernel = {3: "k_inflate_pj", 4: "k_inflate_lanes+k_inflate_resolve"}.get(path, "k_inflate_segments")
    dom = inf_kernel if k_inf >= k_def else "k_deflate_segments"
    kms = max(k_inf, k_def)
    achieved = alg / (kms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(a.traffic_json):
        try:
            tj = json.load(open(a.traffic_json))
            key = f"{a.corpus}:{n}:{a.level}:{dom}"
            traffic = tj.get(key)
        except Exception:
            traffic = None

    if rank == 0:
        res = {
            "metric": "GB/s deflate+inflate on 1 GiB buffer at 1/2/4/8 MI355X; ratio vs reference",
            "value": round(world * n / (ms_step * 1e-3) / 1e9, 4),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": f"deflate level {a.level} + inflate round trip of a {n >> 30} GiB "
                                   f"'{a.corpus}' corpus shard per GPU (SURVEY App. B), device-resident",
                       "corpus": a.corpus, "bytes_per_gpu": n, "level": a.level,
                       "segment_bytes": a.segment, "parallelism": f"shard{world}"},
            "roundtrip_ok": ok,
            "deflate_GBps": round(world * n / (t_def * 1e-3) / 1e9, 4),
            "inflate_GBps": round(world * n / (t_inf * 1e-3) / 1e9, 4),
            "gather_ms": round(t_gat, 4),
            "ratio": round(ratio, 4),
            "ref_ratio": REF_RATIO_L2.get(a.corpus) if a.level == 2 else None,
            "ref_ratio_note": REF_NOTES.get(a.corpus, "reference L2 stream round-trips"),
            "kernel_ms": {"k_deflate_segments": round(k_def, 4), inf_kernel: round(k_inf, 4)},
            "inflate_path": int(recs[-1][4].path),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5),
                         "traffic": traffic, "kernel": dom,
                         "alg_bytes_per_launch": alg,
                         "d2d_copy_GBps": round(d2d_gbps, 1)},
            "cpu_baseline": None,
        }
        if world == 1 and not a.no_cpu_baseline:
            try:
                res["cpu_baseline"] = cpu_baseline(a.corpus, min(a.cpu_sample, n), a.level)
            except Exception as e:  # the baseline is informative, never fatal
                res["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(res), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
