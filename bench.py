"""Headline benchmark: utterances/sec of embedding extraction (80-d FBANK, T=200)
on res2net50_w24_s4_c32 (BASELINE.json configs[2]; the north_star's MFMA
target), one process per GPU, inputs resident in HBM.

A "step" = one forward of one batch of B synthetic utterances through the
whole hot path (input cast -> stem -> 16 Res2Net bottlenecks -> stats-pool ->
BN/dense/BN head); with N > 1 ranks each step also all-gathers the step's
embeddings over RCCL (the cohort assembly of eval_inference_model.sh:38-39).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
       torchrun --nproc-per-node N bench.py --gpus N ...
"""

from __future__ import annotations

import argparse
import io
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3     # f32-input MFMA = vector rate
PEAK_HBM_GBS = 8000.0       # HBM3E spec


def _kernel_name(tag, dt):
    kind = tag & 15
    if tag & (1 << 30):
        return "gemm1x1_ws" if tag & (1 << 17) else "gemm1x1_wide"
    if tag & (1 << 29):
        if tag & (1 << 18):
            if tag & (1 << 17):
                return "conv3x3_utt"
            if tag & (1 << 16):
                return "conv3x3_ks"
            return "conv3x3_s2r" if tag & (1 << 19) else "conv3x3_rw"
        return "conv3x3_pipe"
    if tag & (1 << 28):
        if tag & (1 << 19):
            return "dpn_block_rows"
        return "dpn_down_rows" if tag & (1 << 18) else "gconv3x3_rows"
    if tag & (1 << 27):
        return "gemm1x1_pipe"
    if tag & (1 << 26):
        return "s2_fused" if tag & (1 << 19) else "split_s2_rows"
    if tag & (1 << 25):
        return "chain_fused" if tag & (1 << 19) else "chain_rows"
    if tag & (1 << 24):
        return "bneck_fused"
    if tag & (1 << 23):
        return "conv1x1_smallk" if tag & (1 << 19) else "stem_conv1"
    if tag & (1 << 22):
        return f"split_chain<{(tag >> 4) & 15}, {(tag >> 8) & 15}>"
    if tag & (1 << 21):
        return "conv1x1_nw" if tag & (1 << 19) else "gemm1x1_lds"
    if tag & (1 << 20):
        return f"conv1x1_rr<{(tag >> 16) & 15}, {(tag >> 8) & 15}, {(tag >> 4) & 15}>"
    if tag & (1 << 15):
        return f"conv_win<{(tag >> 4) & 15}, {(tag >> 8) & 15}>"
    if tag & (1 << 14):
        wco, wpx, vec = (tag >> 4) & 15, (tag >> 8) & 15, (tag >> 12) & 1
        t = "float" if tag & (1 << 13) else "__bf16"
        return f"conv_igemm<{t}, {wco}, {wpx}, {'true' if vec else 'false'}>"
    return {1: "stats_pool_k", 2: "splitk_reduce", 3: "other"}.get(kind, "other")


# committed rocprofv3 PMC summaries (tools/pmc_summary.py), one per profiled
# configuration: (model, feat_dim, frames, batch, precision) -> file
PMC_SUMMARIES = {
    ("res2net50_w24_s4_c32", 80, 200, 256, "bf16"): "pmc_summary.json",
    ("tdnn", 80, 200, 64, "bf16"): "pmc_summary_tdnn.json",
    ("dpn68", 80, 600, 64, "bf16"): "pmc_summary_dpn68.json",
}
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_summary.json")


def _load_pmc(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def pmc_traffic(kernel, summ=None):
    """HBM bytes per dispatch of `kernel` from the committed rocprofv3 PMC
    summary (tools/pmc_summary.py: FETCH_SIZE x2 + WRITE_SIZE, the gfx950
    corrections of MI355X_MICROARCH.md "HBM"), averaged over the template
    instances of the same kernel by dispatch count; None if not profiled."""
    if summ is None:
        summ = _load_pmc(PMC_SUMMARY)
    if summ is None:
        return None
    base = kernel.split("<")[0]
    # the stats pool runs as stats_pool_col (short time axis) or stats_pool_k
    bases = {"stats_pool_k", "stats_pool_col"} if base.startswith("stats_pool") else {base}
    tot = disp = 0.0
    for name, r in summ.items():
        if name.split("::")[-1].split("<")[0] in bases and "hbm_bytes" in r:
            n = r["mean"].get("dispatches", 1)
            tot += r["hbm_bytes"] * n
            disp += n
    return tot / disp if disp else None


def pmc_mfma_busy(summ):
    """Conv-stack MFMA utilisation from the PMC summary's MFMA-busy pass:
    SQ_VALU_MFMA_BUSY_CYCLES summed over the kernels with MFMA work against
    1024 SIMDs x their GRBM_GUI_ACTIVE/8 cycles, weighted by dispatches (one
    profiled forward's worth of launches)."""
    if not summ:
        return None
    busy = cyc = 0.0
    per = {}
    for name, r in summ.items():
        m = r.get("mean", {})
        if not m.get("SQ_VALU_MFMA_BUSY_CYCLES") or not r.get("gui_cycles"):
            continue
        n = m.get("dispatches", 1)
        busy += m["SQ_VALU_MFMA_BUSY_CYCLES"] * n
        cyc += 1024.0 * r["gui_cycles"] * n
        per[name.split("(")[0]] = round(r["mfma_busy_frac"], 4)
    return {"conv_stack_mfma_busy": round(busy / cyc, 4) if cyc else None, "per_kernel": per}


def bench_weights(model, feat_dim):
    """(spec, tensors, blob) of the benchmarked network: random-init weights of
    the architecture, BN calibrated on synthetic features (seed 1).  The GPU
    test of the headline plan (tests/test_bf16_oracle.py) uses the same."""
    from voxsrc2020_speaker_verification_amd import archs, synth, weights
    spec = archs.get_arch(model, feat_dim)
    t = synth.make_weights(spec, seed=1)
    buf = io.BytesIO()
    weights.save_blob(buf, spec, t)
    return spec, t, buf.getvalue()


def bench_features(batch, frames, feat_dim, rank=0):
    """The synthetic FBANK batch rank `rank` extracts every step."""
    from voxsrc2020_speaker_verification_amd import synth
    return synth.make_features(batch, frames, feat_dim, seed=1000 + rank)


def weights_blob(model, feat_dim, cache_dir):
    path = os.path.join(cache_dir, f"voxemb_{model}_{feat_dim}_seed1.blob")
    if os.path.exists(path):
        with open(path, "rb") as f:
            return f.read()
    data = bench_weights(model, feat_dim)[2]
    try:
        os.makedirs(cache_dir, exist_ok=True)
        tmp = path + f".{os.getpid()}"
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, path)
    except OSError:
        pass
    return data


def _host_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model, os.cpu_count() or 1


def _cgroup_cpus():
    """CPUs the cgroup's CFS quota grants this process (cgroup v2 cpu.max, or
    v1 cpu.cfs_quota_us / cpu.cfs_period_us), or None when unlimited/unknown.
    A container can see every core in its affinity set and still be capped
    to a few CPUs' worth of time: threads beyond the quota only time-slice."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, int(q) // int(per))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, q // per)
    except (OSError, ValueError):
        pass
    return None


def cpu_baseline(model, feat_dim, T, blob, budget_s=15.0):
    """The C++/OpenMP fp32 restatement of the reference forward
    (oracle/cpu/voxcpu.cpp, the stand-in for tf_extract.py's TF1 CPU
    `sess.run`; kind "port") on a bounded sample of the same workload, on
    every host core this process may run on: its CPU affinity set (SURVEY
    §8(d) "all host cores").  A container can see every core of the host in
    its affinity set and still be capped to a share of them (a cgroup CPU
    quota, or the share the pool announces through OMP_NUM_THREADS): threads
    beyond that only time-slice (on the GPU boxes 256 threads under a 16-CPU
    share ran 6x slower than 16).  So each distinct candidate thread count --
    the affinity count, the cgroup quota, OMP_NUM_THREADS -- is timed on the
    sample and the fastest is the baseline; every trial is recorded."""
    from oracle.cpu import CpuModel, build as cpu_build
    from voxsrc2020_speaker_verification_amd import synth
    cpu_build.build()
    m = CpuModel(blob)
    name, nproc = _host_info()
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = nproc
    quota = _cgroup_cpus()
    omp = os.environ.get("OMP_NUM_THREADS")
    cands = {affinity}
    if quota:
        cands.add(min(quota, affinity))
    if omp and omp.isdigit() and int(omp) > 0:
        cands.add(min(int(omp), affinity))
    cands = sorted(cands)
    per = budget_s / len(cands)
    trials = {}
    best = None
    for threads in cands:
        bs = 2 * threads
        x = synth.make_features(bs, T, feat_dim, seed=99)
        m.run(x[:2], threads)                       # workspace + weights warm
        n, t0 = 0, time.perf_counter()
        while True:
            m.run(x, threads)
            n += bs
            if time.perf_counter() - t0 >= per:
                break
        el = time.perf_counter() - t0
        trials[str(threads)] = round(n / el, 3)
        if best is None or n / el > best[0]:
            best = (n / el, threads, n, el, bs)
    rate, threads, n, el, bs = best
    avx512 = "avx512f" in open("/proc/cpuinfo").read() if os.path.exists("/proc/cpuinfo") else None
    why = (f"fastest of {len(cands)} thread counts tried (affinity {affinity} of {nproc} host cores"
           + (f", cgroup quota {quota}" if quota else "") + (f", OMP_NUM_THREADS {omp}" if omp else "")
           + "; " + ", ".join(f"{k} threads {v} utt/s" for k, v in trials.items()) + ")")
    return {"value": round(rate, 3), "unit": "utterances/sec", "cores": threads, "kind": "port",
            "impl": "cpp_omp", "nproc": nproc, "affinity_cores": affinity,
            "cgroup_cpu_quota": quota, "omp_num_threads_env": omp, "trials": trials,
            "cpu_model": name, "isa": "avx512" if avx512 else "avx2",
            "sample": f"{n} utterances of {T}x{feat_dim} in batches of {bs} ({el:.1f} s; "
                      f"oracle/cpu/voxcpu.cpp fp32 C++/OpenMP, {threads} threads: {why})"}


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` started without a launcher: start N rank processes
    of this same script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one per
    GPU, as torchrun would and as eval_inference_model.sh:29-36 starts
    `num_gpus` tf_extract.py processes) and return the worst exit code.  Runs
    in the parent before anything touches the GPU; the parent never execs."""
    import signal
    import subprocess

    def _term(signum, frame):   # a launcher stopped from outside stops its ranks too
        raise SystemExit(128 + signum)
    signal.signal(signal.SIGTERM, _term)
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    # a rank that fails leaves the others blocked in a collective: stop them
    bad = None
    try:
        while True:
            alive = [p.poll() is None for p in procs]      # poll every rank (no short cut)
            if not any(alive):
                break
            failed = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if failed:
                bad = failed[0]
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
    if bad is None:
        bad = next((p.returncode for p in procs if p.returncode != 0), 0)
    return bad


def stub_rank(args, world, rank):
    """--stub-extractor: the rank/launch logic of main() on the CPU (gloo, a
    numpy stand-in for the forward) so the CPU tests can check that `--gpus N`
    runs N ranks and that the line's n_gpus is the ranks that ran."""
    import torch
    import torch.distributed as dist
    if os.environ.get("VOXEMB_STUB_FAIL_RANK") == str(rank):   # tests: a rank that dies
        raise SystemExit(3)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x = bench_features(2, args.frames, args.feat_dim, rank)
    out = torch.from_numpy(np.concatenate([x.mean(1), x.std(1)], 1).astype(np.float32))
    gathered = [torch.empty_like(out) for _ in range(world)]
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dist.all_gather(gathered, out)
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    pid = torch.tensor([os.getpid()], dtype=torch.int64)
    pids = [torch.zeros_like(pid) for _ in range(world)]
    dist.all_gather(pids, pid)
    if rank == 0:
        print(json.dumps({"metric": "stub", "n_gpus": world,
                          "ranks_ran": len({int(p.item()) for p in pids}), "steps": args.steps,
                          "value": 2 * world * args.steps / max(float(el.item()), 1e-9)}))
    dist.barrier()
    dist.destroy_process_group()


def eer_delta(device, S=64, U=16, T=200, F=80):
    """The metric's "EER delta vs ref" on what the box has (no VoxCeleb, no
    trained graph): synthetic speakers -- a fixed smooth spectral envelope per
    speaker plus per-utterance noise -- through a well-conditioned random-init
    res2net50_w24_s4_c32, the bf16 product path against the fp32 parity path
    (which tests/test_eer_delta.py pins to the C++ oracle), every target pair
    against every non-target pair (tests/test_eer_delta.py: the same task)."""
    import io as _io
    from voxsrc2020_speaker_verification_amd import archs, scoring, synth, weights
    from voxsrc2020_speaker_verification_amd.extractor import Extractor
    spec = archs.get_arch("res2net50_w24_s4_c32", F)
    t = synth.make_weights(spec, seed=1, calib_n=8, calib_T=120, residual_gain=0.25)
    buf = _io.BytesIO()
    weights.save_blob(buf, spec, t)
    rng = np.random.default_rng(2020)
    k = np.exp(-0.5 * (np.arange(-6, 7) / 2.5) ** 2)
    k /= k.sum()
    env = np.stack([np.convolve(e, k, mode="same") for e in rng.standard_normal((S, F))]) * 3
    x = (env[:, None, None, :] + rng.standard_normal((S, U, T, F)) * 1.5).astype(np.float32)
    x = x.reshape(S * U, T, F)
    lab = np.repeat(np.arange(S), U)
    iu = np.triu_indices(S * U, 1)
    y = (lab[iu[0]] == lab[iu[1]]).astype(int)
    res = {}
    for prec in ("bf16", "fp32"):
        with Extractor(buf.getvalue(), device=device, precision=prec) as ex:
            e = ex.run(x)
        e = e / np.linalg.norm(e, axis=1, keepdims=True)
        eer, _, mindcf, _ = scoring.compute_eer_and_min_dcf(y, (e @ e.T)[iu].astype(np.float64))
        res[prec] = (float(eer), float(mindcf))
    return {"task": f"synthetic speakers, {S}x{U} utterances {F}x{T}, well-conditioned "
                    "random-init weights (not VoxCeleb: no data or trained graph here)",
            "target_trials": int(y.sum()), "nontarget_trials": int(len(y) - y.sum()),
            "eer_bf16": round(res["bf16"][0], 6), "eer_fp32_ref": round(res["fp32"][0], 6),
            "delta_eer_abs": round(res["bf16"][0] - res["fp32"][0], 6),
            "mindcf_bf16": round(res["bf16"][1], 5), "mindcf_fp32_ref": round(res["fp32"][1], 5)}


def _progress(msg):
    """A progress line on stderr (stdout carries the one JSON line)."""
    if os.environ.get("RANK", "0") == "0":
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU): without a launcher, N > 1 starts N rank "
                         "processes; under torchrun it must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="res2net50_w24_s4_c32")
    ap.add_argument("--feat-dim", type=int, default=80)
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-eer", action="store_true", help="skip the synthetic-speaker EER delta")
    ap.add_argument("--dump-ops", action="store_true", help="print per-op timing to stderr")
    ap.add_argument("--cache-dir", default=os.environ.get("VOXEMB_CACHE", "/tmp/voxemb_cache"))
    ap.add_argument("--stub-extractor", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            # no launcher: become the launcher (before any GPU call in this process)
            sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE="
              f"{os.environ['WORLD_SIZE']} ranks; refusing to report a line whose n_gpus "
              f"would not be the ranks that ran", file=sys.stderr)
        sys.exit(2)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.stub_extractor:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        return stub_rank(args, world, rank)

    import torch
    import torch.distributed as dist

    # under torchrun (WORLD_SIZE set) the RCCL path runs even at one rank: the
    # per-step all-gather of the embeddings (cohort assembly) is in the timed region
    dist_on = world > 1 or "WORLD_SIZE" in os.environ
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if dist_on else 0)

    from voxsrc2020_speaker_verification_amd.extractor import Extractor

    _progress(f"{args.model} {args.precision}: weights and plan")
    blob = weights_blob(args.model, args.feat_dim, args.cache_dir)
    ex = Extractor(blob, device=dev.index, precision=args.precision)
    B, T, F = args.batch, args.frames, args.feat_dim
    x = torch.from_numpy(bench_features(B, T, F, rank)).to(dev)
    out = torch.empty((B, ex.dim), dtype=torch.float32, device=dev)
    gathered = [torch.empty_like(out) for _ in range(world)] if dist_on else None
    # a dedicated stream (the legacy default stream's handle 0 would make the
    # wrapper fence every step with a side stream, extractor._ordered); the
    # inputs above are complete before it is used
    torch.cuda.synchronize(dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)

    def step():
        ex.run_device(x, out, stream)
        if dist_on:
            dist.all_gather(gathered, out)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist_on:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    ms_per_step = el * 1000.0 / args.steps
    value = world * B * args.steps / el
    _progress(f"timed {args.steps} steps: {ms_per_step:.3f} ms per step")

    # ---- per-kernel timing (HIP events around every launch, same stream)
    prof = ex.profile(x, reps=5, stream=stream)
    if args.dump_ops and rank == 0:
        desc = ex.describe(x)
        for d, ms in zip(desc, prof["ms"]):
            print(f"{ms*1e3:9.1f} us  {d}", file=sys.stderr)
    groups = {}
    for ms, fl, by, tag in zip(prof["ms"], prof["flops"], prof["bytes"], prof["kind"]):
        g = groups.setdefault(_kernel_name(int(tag), args.precision),
                              {"ms": 0.0, "flops": 0.0, "bytes": 0.0, "n": 0, "kind": int(tag) & 15})
        g["ms"] += float(ms)
        g["flops"] += float(fl)
        g["bytes"] += float(by)
        g["n"] += 1
    # the conv stack: every backbone kernel with MFMA work (not the fp32 head)
    conv = {k: v for k, v in groups.items() if v["flops"] > 0 and v["kind"] == 0}
    dom_name, dom = max(conv.items(), key=lambda kv: kv[1]["ms"])
    peak = PEAK_F32_TFLOPS if "float" in dom_name else PEAK_BF16_TFLOPS
    ach = (dom["flops"] / dom["n"]) / (dom["ms"] / dom["n"] * 1e-3) / 1e12
    # which roof bounds the dominant kernel: the larger of its FLOP time at the
    # dense MFMA peak and its algorithmic-byte time at the HBM peak (the 1x1
    # GEMMs at B=256 are 70-440 FLOP/B against a machine balance of ~310)
    t_mfma = dom["flops"] / (peak * 1e12)
    t_hbm = dom["bytes"] / (PEAK_HBM_GBS * 1e9)
    ach_gbs = (dom["bytes"] / dom["n"]) / (dom["ms"] / dom["n"] * 1e-3) / 1e9
    fwd_ms = float(np.sum(prof["ms"]))
    conv_fl = sum(v["flops"] for v in conv.values())
    conv_ms = sum(v["ms"] for v in conv.values())
    pool = groups.get("stats_pool_k")
    # the committed PMC summary was collected on the default workload only; on any
    # other model/shape its per-launch bytes belong to different launches
    pmc_file = PMC_SUMMARIES.get((args.model, F, T, B, args.precision))
    summ = _load_pmc(os.path.join(ROOT, "profiles", pmc_file)) if pmc_file else None
    traffic = (lambda k: pmc_traffic(k, summ)) if summ else (lambda k: None)
    if t_hbm >= t_mfma:
        roof = {"bound": "hbm", "kernel": dom_name, "launches_per_step": dom["n"],
                "achieved": round(ach_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(ach_gbs / PEAK_HBM_GBS, 4)}
    else:
        roof = {"bound": "mfma", "kernel": dom_name, "launches_per_step": dom["n"],
                "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(ach / peak, 4)}
    roof.update({
        "traffic": traffic(dom_name),
        "traffic_unit": f"HBM bytes per launch (rocprofv3 PMC, profiles/{pmc_file})",
        "algorithmic_bytes_per_launch": dom["bytes"] / dom["n"],
        "algorithmic_bytes_def": "input pixels sampled + output (+ residual) once, bf16, plus the "
                                 "weights once per XCD (8 L2s)",
        "avg_launch_us": round(dom["ms"] / dom["n"] * 1e3, 2),
        "flop_per_launch": dom["flops"] / dom["n"],
        "mfma_tflops": round(ach, 2), "mfma_frac": round(ach / peak, 4),
        "hbm_gbs": round(ach_gbs, 1), "hbm_frac": round(ach_gbs / PEAK_HBM_GBS, 4),
        # fraction of the kernel's own roofline time max(FLOP/peak, bytes/BW)
        "roofline_frac": round(max(t_mfma, t_hbm) / (dom["ms"] * 1e-3), 4)})
    extra = {
        "conv_stack": {"achieved_tflops": round(conv_fl / (conv_ms * 1e-3) / 1e12, 2),
                       "frac": round(conv_fl / (conv_ms * 1e-3) / 1e12 / peak, 4),
                       "ms": round(conv_ms, 3), "flop": conv_fl},
        "mfma_pmc": (dict(pmc_mfma_busy(summ) or {}, source=f"profiles/{pmc_file}")
                     if summ else None),
        "forward_ms_profiled": round(fwd_ms, 3),
        "kernels": {k: {"n": v["n"], "ms": round(v["ms"], 4),
                        "tflops": round(v["flops"] / max(v["ms"], 1e-9) / 1e9, 2) if v["flops"] else None,
                        "gbs": round(v["bytes"] / max(v["ms"], 1e-9) / 1e6, 1)}
                    for k, v in sorted(groups.items(), key=lambda kv: -kv[1]["ms"])},
    }
    if pool:
        gbs = pool["bytes"] / pool["n"] / (pool["ms"] / pool["n"] * 1e-3) / 1e9
        extra["stats_pool_roofline"] = {"bound": "hbm", "achieved": round(gbs, 1),
                                        "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                        "frac": round(gbs / PEAK_HBM_GBS, 4),
                                        "traffic": traffic("stats_pool_k"),
                                        "bytes_per_launch": pool["bytes"] / pool["n"]}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        _progress("CPU baseline (bounded sample) and the fp32 like-for-like line")
        cpu = cpu_baseline(args.model, F, T, blob)
        # like for like: the CPU baseline computes in fp32, the headline in bf16;
        # the same workload through the GPU's fp32 path, a few timed steps
        if args.precision == "bf16":
            ex32 = Extractor(blob, device=dev.index, precision="fp32")
            out32 = torch.empty((B, ex32.dim), dtype=torch.float32, device=dev)
            ex32.run_device(x, out32, stream)
            torch.cuda.synchronize(dev)
            n32, t32 = 10, time.perf_counter()
            for _ in range(n32):
                ex32.run_device(x, out32, stream)
            torch.cuda.synchronize(dev)
            v32 = B * n32 / (time.perf_counter() - t32)
            ex32.close()
            cpu["gpu_fp32_same_workload"] = {
                "value": round(v32, 1), "unit": "utterances/sec", "steps": n32,
                "ratio_to_cpu": round(v32 / cpu["value"], 2),
                "note": "the timed workload through the GPU's fp32 path (the CPU baseline's "
                        "precision); the bf16 line's ratio is ratio_bf16_to_cpu"}
            cpu["ratio_bf16_to_cpu"] = round(value / cpu["value"], 2)

    eer = None
    # beside the CPU baseline (both reference comparisons; the profiling runs pass
    # --no-cpu-baseline and so keep their dispatch lists to the timed workload)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.no_eer \
            and args.model == "res2net50_w24_s4_c32" and args.precision == "bf16":
        _progress("synthetic-speaker EER delta")
        eer = eer_delta(dev.index, F=F)

    if rank == 0:
        line = {
            "metric": "utterances/sec (80-d FBANK, T=200) embedding extraction",
            "value": round(value, 1), "unit": "utterances/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.precision, "data": "synthetic (seeded N(0,1) FBANK, random-init "
                                            "calibrated weights)",
            "config": {"workload": f"{args.model} {F}x{T} extraction", "global_batch": B * world,
                       "per_gpu_batch": B, "frames": T, "feat_dim": F,
                       "parallelism": f"dp{world}" + (" + RCCL all-gather" if dist_on else "")},
            "roofline": roof,
            "cpu_baseline": cpu,
            "eer_delta_vs_fp32": eer,
            **extra,
        }
        print(json.dumps(line))
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()
    ex.close()


if __name__ == "__main__":
    main()
