"""Benchmark of the `aln` hot path (BASELINE.json metric: query residues aligned/s,
bit-identical hits). Workload = BASELINE.json configs[3] on one GPU per rank:
synthetic 1M queries (avg ~265 aa before the 127-residue cap, L = 127) against a
10M-residue DB, default `aln` options (BLOSUM62 11/1, -b 10, -r 16, -t 2, -s 2).

    python bench.py [--gpus N --steps K --warmup W] [--queries 1000000]
                    [--db-residues 10000000] [--cpu-sample 2000] [--no-cpu]

A step = one full `aln` pass over the rank's query set with inputs resident in HBM:
K1 seed -> K2 score -> host merge -> K3 traceback -> E-values + text formatting
(in memory) -> (N > 1) RCCL gather of the 32-byte hit records to rank 0.
Multi-GPU: one process per GPU (torchrun); each rank searches its own 1M-query
shard (weak scaling), hit records are gathered to rank 0 over RCCL.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_VALU_TOPS = 78.6   # 256 CU x 4 SIMD x 32 lanes/cycle x 2.4 GHz int32 ops (MI355X_MICROARCH.md)
PEAK_VALU_PK16_TOPS = 157.3  # the same issue rate, two 16-bit ops per lane (v_pk_*_u16/i16)
PEAK_HBM_GBS = 8000.0   # HBM3E spec
SCORE_OPS_PER_CELL = 10  # Gotoh cell: add, max3 (H), add (open), add+max (E), add+max (F), max (colmax)


PAM250 = os.path.join(REPO, "tests", "golden", "matrices", "PAM250")
# BASELINE.json configs: synthetic data, splitmix64 seeds 3/4/5
PRESETS = {
    "cfg4": {"queries": 1_000_000, "db": 10_000_000, "seed": 4, "aln": [],
             "workload": "cfg4: synthetic 1M queries (avg 300 aa requested, L=127) x 10M-residue DB, per rank"},
    "cfg3": {"queries": 100_000, "db": 5_000_000, "seed": 3, "aln": [],
             "workload": "cfg3: synthetic 100k queries (L=127) x 5M-residue DB, per rank"},
    "cfg5": {"queries": 100_000, "db": 5_000_000, "seed": 5, "aln": ["-r", "64", "-M", PAM250, "-y", "2"],
             "workload": "cfg5: wide band -r 64, PAM250 11/1, -y 2; synthetic 100k queries x 5M-residue DB"},
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_data(root: str, nq: int, db_res: int, first: int, seed: int = 4) -> None:
    ghostm = os.path.join(REPO, "ghostm_amd", "bin", "ghostm")
    os.makedirs(root, exist_ok=True)
    run = lambda *a: subprocess.run([ghostm, *a], check=True, stdout=subprocess.DEVNULL,  # noqa: E731
                                    stderr=subprocess.DEVNULL)
    run("synth", "-d", f"{root}/db.fa", "-q", f"{root}/q.fa", "-n", str(nq), "-N", str(db_res),
        "-s", str(seed), "-f", str(first))
    run("db", "-i", f"{root}/db.fa", "-o", f"{root}/db")
    run("qry", "-i", f"{root}/q.fa", "-o", f"{root}/q", "-l", "300")
    os.remove(f"{root}/q.fa")


def cpu_baseline(root: str, nsample: int, db_res: int, first: int, seed: int = 4,
                 aln_args: list | None = None) -> dict:
    """The reference's own CPU path (oracle/_ref/ghostm_ref: GHOSTM's aligner.cpp
    compiled from the reference sources, run without -D) on the first `nsample`
    queries of this rank's workload against the same DB, single-threaded as the
    reference is. Falls back to this repo's CPU restatement (oracle/ghostm_oracle)
    when the reference build is absent. Also checks that the GPU output on that
    sample is byte-identical to the CPU program's."""
    ghostm = os.path.join(REPO, "ghostm_amd", "bin", "ghostm")
    ref = os.path.join(REPO, "oracle", "_ref", "ghostm_ref")
    port = os.path.join(REPO, "oracle", "_build", "ghostm_oracle")
    use_ref = os.path.exists(ref)
    exe = ref if use_ref else port
    sub = os.path.join(root, "sample")
    os.makedirs(sub, exist_ok=True)
    subprocess.run([ghostm, "synth", "-q", f"{sub}/q.fa", "-n", str(nsample), "-N", str(db_res),
                    "-s", str(seed), "-f", str(first)], check=True, capture_output=True)
    subprocess.run([ghostm, "qry", "-i", f"{sub}/q.fa", "-o", f"{sub}/q", "-l", "300"], check=True,
                   capture_output=True)
    t0 = time.perf_counter()
    subprocess.run([exe, "aln", "-i", f"{sub}/q", "-d", f"{root}/db", "-o", f"{sub}/cpu.out"]
                   + list(aln_args or []), check=True, capture_output=True)
    dt = time.perf_counter() - t0
    from ghostm_amd.aligner import Session

    with Session(["-i", f"{sub}/q", "-d", f"{root}/db", "-o", f"{sub}/gpu.out", "-D", str(_device())]
                 + list(aln_args or [])) as s:
        s.run()
        gpu = s.output()
        residues = s.stats()["query_residues"]
    same = gpu == open(f"{sub}/cpu.out", "rb").read()
    what = ("reference aligner.cpp CPU path (oracle/_ref/ghostm_ref, reference sources, g++ -O2)" if use_ref
            else "CPU restatement (oracle/ghostm_oracle.cpp, g++ -O2)")
    return {"value": residues / dt, "unit": "query residues/s", "cores": 1,
            "kind": "reference" if use_ref else "port",
            "sample": f"first {nsample} queries of rank 0's workload vs the same {db_res / 1e6:g}M-residue DB "
                      f"({residues} residues, {dt:.1f} s, {what}, 1 thread)",
            "bit_identical_to_gpu_on_sample": bool(same), "residues": residues}


def cpu_baseline_multi(root: str, nsample: int, db_res: int, first: int, residues: int, seed: int = 4,
                       aln_args: list | None = None, procs: int | None = None) -> dict | None:
    """SURVEY §8 d4's second CPU figure: the same sample on all host cores the job
    may use. The reference aligner is single-threaded, so it runs as `procs`
    processes over contiguous query ranges (queries are independent; the
    concatenated outputs must equal the one-process output, checked here)."""
    ref = os.path.join(REPO, "oracle", "_ref", "ghostm_ref")
    port = os.path.join(REPO, "oracle", "_build", "ghostm_oracle")
    exe = ref if os.path.exists(ref) else port
    ghostm = os.path.join(REPO, "ghostm_amd", "bin", "ghostm")
    # the box's CPU share is 16 (OMP_NUM_THREADS is set to it); os.cpu_count()
    # there reports the whole machine
    procs = procs or max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)),
                                os.cpu_count() or 1))
    sub = os.path.join(root, "sample")
    parts = []
    per = (nsample + procs - 1) // procs
    for k in range(procs):
        n = min(per, nsample - k * per)
        if n <= 0:
            break
        d = os.path.join(sub, f"part{k}")
        os.makedirs(d, exist_ok=True)
        subprocess.run([ghostm, "synth", "-q", f"{d}/q.fa", "-n", str(n), "-N", str(db_res), "-s", str(seed),
                        "-f", str(first + k * per)], check=True, capture_output=True)
        subprocess.run([ghostm, "qry", "-i", f"{d}/q.fa", "-o", f"{d}/q", "-l", "300"], check=True,
                       capture_output=True)
        parts.append(d)
    t0 = time.perf_counter()
    running = [subprocess.Popen([exe, "aln", "-i", f"{d}/q", "-d", f"{root}/db", "-o", f"{d}/cpu.out"]
                                + list(aln_args or []), stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
               for d in parts]
    rcs = [p.wait() for p in running]
    dt = time.perf_counter() - t0
    if any(rcs):
        return None
    joined = b"".join(open(f"{d}/cpu.out", "rb").read() for d in parts)
    single = open(f"{sub}/cpu.out", "rb").read()
    return {"value": residues / dt, "unit": "query residues/s", "cores": len(parts),
            "kind": "reference" if exe == ref else "port",
            "sample": f"the cpu_baseline sample as {len(parts)} processes over contiguous query ranges "
                      f"({dt:.1f} s)",
            "identical_to_one_process": joined == single}


def _device() -> int:
    # GHOSTM_BENCH_DEVICE pins every rank to one device (rehearsing the
    # multi-rank path on a one-GPU machine)
    return int(os.environ.get("GHOSTM_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))


def load_pmc_traffic() -> dict | None:
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--preset", choices=sorted(PRESETS), default="cfg4",
                    help="BASELINE.json config (cfg4 = the headline workload)")
    ap.add_argument("--queries", type=int, default=None, help="queries per rank (default: preset)")
    ap.add_argument("--db-residues", type=int, default=None)
    ap.add_argument("--cpu-sample", type=int, default=2000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--aln", default="", help="extra aln options appended to the preset's (e.g. '-l 64')")
    args = ap.parse_args()
    preset = PRESETS[args.preset]
    if args.queries is None:
        args.queries = preset["queries"]
    if args.db_residues is None:
        args.db_residues = preset["db"]
    aln_args = list(preset["aln"]) + args.aln.split()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(_device())
        # RCCL ("nccl") over xGMI; GHOSTM_BENCH_BACKEND=gloo rehearses the same
        # calls on a one-GPU machine (RCCL refuses two ranks on one device)
        backend = os.environ.get("GHOSTM_BENCH_BACKEND", "nccl")
        dist.init_process_group(backend)
        coll_dev = "cuda" if backend == "nccl" else "cpu"
    from ghostm_amd.aligner import Session

    workdir = args.workdir or tempfile.mkdtemp(prefix=f"ghostm_bench_r{rank}_")
    t0 = time.perf_counter()
    first = rank * args.queries
    make_data(workdir, args.queries, args.db_residues, first, seed=preset["seed"])
    log(f"[rank {rank}] data ready in {time.perf_counter() - t0:.1f}s at {workdir}")
    sess = Session(["-i", f"{workdir}/q", "-d", f"{workdir}/db", "-o", f"{workdir}/out", "-D", str(_device())]
                   + aln_args)

    def step():
        sess.run()
        if dist is not None:
            from ghostm_amd.aligner import HIT_DTYPE
            from ghostm_amd.shard import gather_device_records

            merged = gather_device_records(sess.device_hits().to(coll_dev), dist, HIT_DTYPE.itemsize)
            if rank == 0:
                step.gathered = sum(m.numel() for m in merged) // HIT_DTYPE.itemsize
    step.gathered = 0

    for _ in range(args.warmup):
        step()

    def sync():
        if dist is not None:
            import torch

            dist.barrier()
            torch.cuda.synchronize()

    sync()
    t = time.perf_counter()
    st_acc = None
    for _ in range(args.steps):
        step()
        st = sess.stats()
        if st_acc is None:
            st_acc = {k: 0 for k in st}
        for k, v in st.items():
            st_acc[k] += v
    sync()
    elapsed = time.perf_counter() - t
    if dist is not None:
        import torch

        e = torch.tensor([elapsed], device=coll_dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
        res = torch.tensor([st_acc["query_residues"]], device=coll_dev, dtype=torch.float64)
        dist.all_reduce(res)
        total_res = float(res.item())
    else:
        total_res = float(st_acc["query_residues"])

    k = args.steps
    per = {key: v / k for key, v in st_acc.items()}
    cpu = cpu_multi = None
    if rank == 0 and world == 1 and not args.no_cpu:  # the CPU baseline is an N=1 figure
        cpu = cpu_baseline(workdir, args.cpu_sample, args.db_residues, first, preset["seed"], aln_args)
        cpu_multi = cpu_baseline_multi(workdir, args.cpu_sample, args.db_residues, first,
                                       cpu.pop("residues"), preset["seed"], aln_args)
    if rank == 0:
        score_t = per["seconds_score"] / max(1, per["score_launches"])
        score_cells = per["score_cells"] / max(1, per["score_launches"])
        achieved = score_cells * SCORE_OPS_PER_CELL / score_t / 1e12 if score_t > 0 else 0.0
        packed = per["score_launches_packed"] == per["score_launches"] and per["score_launches"] > 0
        half = packed and per["score_launches_half"] == per["score_launches"]
        peak = PEAK_VALU_PK16_TOPS if packed else PEAK_VALU_TOPS
        framed = half and per.get("score_launches_framed", 0) == per["score_launches"]
        if framed:
            kname = ("k_score16f<32> (K2 Gotoh DP, packed f16 holding exact integers in a per-column frame, "
                     "two candidates per lane)")
        elif half:
            kname = "k_score16<32,f16> (K2 Gotoh DP, packed f16 holding exact integers, two candidates per lane)"
        elif packed:
            kname = "k_score16<32,int16> (K2 Gotoh DP, packed int16, two candidates per lane)"
        else:
            kname = "k_score (K2 Gotoh DP, int32)"
        dtype = "f16" if half else ("int16" if packed else "int32")
        pmc = load_pmc_traffic()
        traffic = None
        if pmc and pmc.get("queries") == args.queries:
            traffic = pmc.get("k_score_hbm_bytes_per_launch")
        seed_gbs = per["seed_bytes"] / per["seconds_seed"] / 1e9 if per["seconds_seed"] > 0 else 0.0
        out = {
            "metric": "query residues aligned/sec (whole node) + bit-identical hit-list vs CPU",
            "value": total_res / elapsed,
            "unit": "query residues/s",
            "n_gpus": world,
            "steps": k,
            "warmup": args.warmup,
            "ms_per_step": elapsed / k * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dtype,
            "data": f"synthetic (ghostm synth, splitmix64 seed {preset['seed']}; "
                    f"aln options {' '.join(aln_args) if aln_args else 'defaults (BLOSUM62 11/1)'})",
            "config": {
                "workload": preset["workload"],
                "aln_options": aln_args,
                "queries_per_rank": args.queries,
                "db_residues": args.db_residues,
                "query_residues_per_rank_step": per["query_residues"],
                "candidates_per_rank_step": per["candidates"],
                "hits_per_rank_step": per["hits"],
                "parallelism": f"query-shard x{world} (one process per GPU, RCCL gather of hit records)",
            },
            "roofline": {
                "bound": "valu",
                "kernel": kname,
                "achieved": achieved,
                "peak": peak,
                "unit": "Tops/s",
                "frac": achieved / peak,
                "traffic": traffic,
                "cells_per_launch": score_cells,
                "ops_per_cell": SCORE_OPS_PER_CELL,
                "gcups": score_cells / score_t / 1e9 if score_t > 0 else 0.0,
                "avg_launch_ms": score_t * 1e3,
            },
            "roofline_hbm": {
                "bound": "hbm",
                "kernel": "K1 seed stage per step (k_seed_lists, k_seed_hash, k_compact: gathers of CSR positions)",
                "achieved": seed_gbs,
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": seed_gbs / PEAK_HBM_GBS,
                "algorithmic_bytes_per_step": per["seed_bytes"],
                "traffic": pmc.get("k1_hbm_bytes_per_step") if (pmc and pmc.get("queries") == args.queries) else None,
            },
            "stages_s_per_step": {
                "total": per["seconds_total"],
                "seed_device": per["seconds_seed"],
                "score_device": per["seconds_score"],
                "traceback_device": per["seconds_traceback"],
                "merge_host": per["seconds_merge"],
                "output_host": per["seconds_output"],
            },
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_multi,
        }
        print(json.dumps(out), flush=True)
    sess.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if not args.workdir:
        shutil.rmtree(workdir, ignore_errors=True)


if __name__ == "__main__":
    main()
