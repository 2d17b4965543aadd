#!/usr/bin/env python
"""Headline benchmark: % partitions verified + partitions/s on the AC suite (BASELINE.json).

Workload = the reference's ``src/AC`` experiment (Table V of the paper): the 12 Adult-census
MLP architectures AC-1..AC-12, the full 16 000-partition grid per model (partition size 10),
protected attribute ``sex``, 1 000 simulation points per partition, heuristic retry on
UNKNOWN (HEURISTIC_PRUNE_THRESHOLD 5).  One *step* = verify the whole suite grid
(192 000 partitions) once; with N GPUs the seeded partition order is sharded across the N
ranks (strong scaling: total work fixed).  Weights are random-init (glorot-uniform, fixed
seed) per BASELINE.json; ``--weights zoo`` uses the reference's trained weights instead.

value  = SOUNDLY decided partitions per second, whole job: SAT pairs confirmed exactly on the
         original network + UNSAT from rigorous proofs (stages bab / relu / beta / lp / smt).
         Heuristic-retry UNSAT (the reference's unsound retry, src/AC/Verify-AC.py:173-212), a
         trusted MILP's floating-point UNSAT and heuristic SAT pairs that do not flip the
         original network are excluded; the all-verdict rate the reference would count is the
         secondary field ``decided_per_s_all``.
vs_baseline = value / 0.02497 decided partitions/s, the reference's AC/sex aggregate from
Table V (553 decided in sum(#P x Total) = 22 144 s).  That reference number is on
its TRAINED weights; this bench runs random-init weights of the same shapes (BASELINE.json).  The
trained-weight Table-V comparison is a separate run (tools/baseline_configs.py, README), not a
field of this line.

JSON keys (rank 0 prints one line; tests/test_bench_launch.py checks every one is present):
metric, value, unit, n_gpus, steps, warmup, ms_per_step, higher_is_better, scaling, vs_baseline,
dtype, data, config, decided_per_s_all, pct_verified, pct_verified_sound, partitions_per_s, sat,
unsat, unknown, unsat_sound, unsat_heuristic, sat_by_stage, unsat_by_stage, dist, baseline,
vs_baseline_note, per_model.

Multi-GPU: one process per GPU, ``torch.distributed`` backend ``nccl`` (= RCCL over xGMI).

    python bench.py --gpus 1 --steps 1 --warmup 1
    python bench.py --gpus 8                      # self-launches 8 ranks (no torchrun needed)
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8 --steps 1 --warmup 1

Self-launch: with ``--gpus N > 1`` and no ``WORLD_SIZE`` in the environment, this process
starts N child processes of itself (rank env vars set, rendezvous on 127.0.0.1) BEFORE any GPU
call, waits for them and exits with their worst return code; rank 0 prints the JSON line.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_DECIDED_PER_S = 553.0 / 22143.5
METRIC = "% partitions verified + partitions/sec on AC suite at 1/2/4/8 MI355X"
STAGES = ("sim", "bab", "relu", "beta", "lp", "falsify", "smt", "milp", "heuristic", "heuristic-confirmed")
UNSOUND_UNSAT = ("heuristic", "milp")     # engine/stages.py: UNSAT verdicts that are not proofs


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--preset", default="src/AC-sex")
    ap.add_argument("--weights", default="random", choices=["random", "zoo"])
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--scope", default="suite", choices=["suite", "chunk"],
                    help="suite: one step = whole grid of every model (strong scaling); "
                         "chunk: one step = --chunk partitions per model per rank (weak scaling)")
    ap.add_argument("--chunk", type=int, default=0,
                    help="partitions per work item; 0 = by shard size: 8192 when a rank holds more than 8192 "
                         "partitions per model (N=1: two 8000-partition items per model), else 4096 "
                         "(profiles/r2/s4/chunk/)")
    ap.add_argument("--limit", type=int, default=0,
                    help="verify only the first LIMIT partitions of the seeded order per model (tests)")
    ap.add_argument("--node-budget", type=int, default=512)
    ap.add_argument("--heuristic-node-budget", type=int, default=512,
                    help="BaB node budget of the heuristic retry on the pruned network")
    ap.add_argument("--escalate-budget", type=int, default=32768,
                    help="second sound BaB pass with this node budget on the first pass's UNKNOWN residue")
    ap.add_argument("--escalate-max-open", type=int, default=384,
                    help="escalate only partitions that left <= this many open BaB nodes (0 = all)")
    ap.add_argument("--escalate-probation", default="2048:768,4096:768,8192:768,16384:1024",
                    help="intermediate inline-escalation steps 'budget:max_open,...' between --node-budget and "
                         "--escalate-budget")
    ap.add_argument("--stages", default="",
                    help="further escalation passes 'budget:max_open,...' after --escalate-budget")
    ap.add_argument("--relu-budget", type=int, default=1024,
                    help="ReLU-phase BaB (stage 'relu') on the input-split residue: nodes per partition (0 = off)")
    ap.add_argument("--relu-max-width", type=int, default=16,
                    help="run the relu stage only on networks whose hidden layers are at most this wide")
    ap.add_argument("--relu-escalate-cap", type=int, default=2048,
                    help="models the relu stage runs on: cap the input-split escalation budget (0 = no cap)")
    ap.add_argument("--beta-budget", type=int, default=0,
                    help="beta-CROWN phase-split BaB (stage 'beta') in the fixed passes: nodes per partition "
                         "(0 = only in the budget pass's anytime rounds).  On this random-init suite its "
                         "fixed-pass yield is ~60 verdicts per step for +350-420 ms (profiles/r5/bench_ab); on "
                         "trained nets it decides the residue (profiles/r5/ac7_trained)")
    ap.add_argument("--batch-nodes", type=int, default=65536,
                    help="BaB nodes bounded per sub-batch launch (memory per runtime scales with it)")
    ap.add_argument("--smt", default="none",
                    help="exact host solver on the residue in the timed steps: none (fixed-budget throughput "
                         "bench) | auto | milp | z3py | z3bin")
    ap.add_argument("--trust-milp", action="store_true",
                    help="count a HiGHS MILP 'unsat' (floating-point dual bound) as an UNSAT verdict (stage "
                         "'milp', excluded from the sound figures); default: recorded, partition stays UNKNOWN")
    ap.add_argument("--lp-budget", type=int, default=4096,
                    help="with --smt milp/auto: verified-LP branch-and-bound nodes per partition (stage 'lp', "
                         "sound UNSAT); 0 = the HiGHS MILP")
    ap.add_argument("--budget-pass", type=float, default=10.0,
                    help="after the timed steps, one untimed pass over the same grid in anytime mode with this "
                         "many seconds per model (growing BaB budgets + falsifier + MILP rounds on the residue): "
                         "reports pct_verified_at_budget (0 = skip; default 10 s per model adds ~16 s)")
    ap.add_argument("--no-heuristic", action="store_true",
                    help="skip the reference's unsound heuristic retry (sound verdicts only)")
    ap.add_argument("--residual-samples", type=int, default=None, help="residual falsifier samples (0 = off)")
    ap.add_argument("--residual-iters", type=int, default=None)
    ap.add_argument("--bisect-steps", type=int, default=None, help="boundary-walk bisection steps (0 = off)")
    ap.add_argument("--sim-size", type=int, default=None)
    ap.add_argument("--models", default=None, help="comma list (default: the preset's models)")
    ap.add_argument("--device", default=None)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--emulate-shard", default=None,
                    help="r/N: run only rank r's shard of an N-rank job on this one process (diagnostics)")
    ap.add_argument("--priority-items", type=int, default=0,
                    help="run the N heaviest items of a step (previous step's wall time) on high-priority "
                         "HIP streams (0 = off)")
    ap.add_argument("--profile", action="store_true", help="per-stage timing breakdown on stderr (syncs)")
    ap.add_argument("--concurrency", type=int, default=0,
                    help="host threads / HIP streams verifying (model, chunk) items concurrently (default: the "
                         "rank's CPUs, at most 8, on GPU)")
    ap.add_argument("--unit", type=int, default=250,
                    help="N > 1: partitions per load-balancing unit (LPT over ranks on the previous step's BaB node "
                         "counts; parallel/balance.py)")
    ap.add_argument("--no-balance", action="store_true",
                    help="N > 1: the strided shard of round 2 instead of the LPT unit assignment")
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(args) -> int:
    """Start ``--gpus`` ranks of this script (one per GPU) and wait for them.

    This process never touches the GPU (no torch import at all), so its children start from a
    clean HIP state; each child binds ``cuda:LOCAL_RANK`` and joins the RCCL group."""
    n = args.gpus
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FAIRIFY_BENCH_CHILD="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def _native_mem():
    try:
        from fairify_amd.ops import ext

        return dict(ext().mem_stats())
    except Exception:
        return None


def _mem_delta(a, b):
    if not a or not b:
        return None
    return {"driver_frees": b["driver_frees"] - a["driver_frees"], "dev_mallocs": b["dev_mallocs"] - a["dev_mallocs"],
            "dev_cache_hits": b["dev_hits"] - a["dev_hits"], "host_mallocs": b["host_mallocs"] - a["host_mallocs"],
            "dev_gb": round((b["dev_live_bytes"] + b["dev_cached_bytes"]) / 2 ** 30, 3),
            "host_pinned_gb": round((b.get("host_live_bytes", 0) + b.get("host_cached_bytes", 0)) / 2 ** 30, 3)}


def main() -> None:
    args = parse_args()
    if os.environ.get("FAIRIFY_FORCE_REFERENCE") == "1":
        raise SystemExit("bench.py refuses FAIRIFY_FORCE_REFERENCE=1: the benchmark must run the HIP kernels")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and not args.emulate_shard:
        raise SystemExit(launch(args))
    # one node runs LOCAL_WORLD_SIZE ranks: each takes its own slice of the host CPUs for its host
    # threads / HIP streams / MILP pool, pinned before anything touches the GPU (self-launch and
    # torchrun alike; FAIRIFY_NO_PIN=1 disables it)
    from fairify_amd.parallel import balance as BL

    lw = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    if args.emulate_shard and lw <= 1:
        # one rank of an N-rank node on this process: its CPU slice too
        cpus = BL.pin_rank(*(int(v) for v in args.emulate_shard.split("/")))
    else:
        cpus = BL.pin_rank(int(os.environ.get("LOCAL_RANK", "0")), lw)

    import torch

    from fairify_amd import presets
    from fairify_amd.engine.pipeline import VerifyConfig, verify_chunk
    from fairify_amd.models.zoo import get_model
    from fairify_amd.ops.backend import Backend
    from fairify_amd.parallel import dist as D
    from fairify_amd.partition import processing_order
    from fairify_amd.utils.timer import StageTimer

    dev_type = args.device or ("cuda" if torch.cuda.device_count() > 0 else "cpu")
    info = D.init(dev_type)
    if dev_type == "cpu":      # CPU rehearsal ranks share the host's cores; FAIRIFY_CPU_THREADS pins the
        # intra-op thread count (CPU matmul summation order depends on it, and bounds at a decision
        # threshold may flip: tests comparing rank counts pin it)
        nt = os.environ.get("FAIRIFY_CPU_THREADS")
        if nt or info.world > 1:
            torch.set_num_threads(int(nt) if nt else max(1, (os.cpu_count() or 1) // info.world))
    if not args.emulate_shard and info.world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={info.world}: launch one rank per GPU")
    if dev_type == "cuda" and info.world > torch.cuda.device_count() and \
            os.environ.get("FAIRIFY_DIST_BACKEND", "nccl") == "nccl":
        raise SystemExit(f"{info.world} ranks but only {torch.cuda.device_count()} GPUs visible")
    backend_name = D.backend_name(info)
    pre = presets.get(args.preset)
    grid = pre.grid()
    q = pre.resolved()
    order = processing_order(grid, seed=args.seed)
    if args.limit:
        order = order[:args.limit]
    shard = order[info.rank::info.world]
    if args.emulate_shard:
        er, en = (int(v) for v in args.emulate_shard.split("/"))
        shard = order[er::en]
    if args.chunk <= 0:
        # big items make big launches; below 8192 partitions per model a second item per model
        # beats a bigger one (N=1: 8192 1 237-1 265 ms vs 4096 1 285-1 328 ms; half shard: 4096
        # 645 ms vs 8192 692-711 ms)
        args.chunk = 8192 if len(shard) > 8192 else 4096
    names = args.models.split(",") if args.models else list(pre.models)
    models = [get_model(n, weights=args.weights, seed=args.seed) for n in names]
    backends = [Backend(m, device=info.device) for m in models]
    if info.device.type == "cuda" and not all(be.hip for be in backends):
        raise SystemExit("HIP extension inactive on a GPU run")
    cfg = VerifyConfig(sim_size=args.sim_size or pre.sim_size, seed=args.seed, chunk=args.chunk,
                       soft_timeout=pre.soft_timeout, hard_timeout=pre.hard_timeout,
                       node_budget=args.node_budget, heuristic=not args.no_heuristic, heuristic_p=pre.heuristic_p,
                       heuristic_node_budget=args.heuristic_node_budget, escalate_budget=args.escalate_budget,
                       escalate_max_open=args.escalate_max_open, batch_nodes=args.batch_nodes,
                       smt_backend=args.smt, trust_milp=args.trust_milp, lp_budget=args.lp_budget, relu_budget=args.relu_budget,
                       relu_max_width=args.relu_max_width, relu_escalate_cap=args.relu_escalate_cap,
                       beta_budget=args.beta_budget,
                       escalate_probation=tuple(tuple(int(v) for v in st.split(":"))
                                                for st in args.escalate_probation.split(",") if st),
                       escalate_stages=tuple(tuple(int(v) for v in st.split(":")) for st in args.stages.split(",") if st))
    if args.residual_samples is not None:
        cfg.residual_samples = args.residual_samples
    if args.residual_iters is not None:
        cfg.residual_iters = args.residual_iters
    if args.bisect_steps is not None:
        cfg.bisect_steps = args.bisect_steps

    def chunks_for_step(step: int):
        if args.scope == "suite":
            return [shard[s:s + args.chunk] for s in range(0, len(shard), args.chunk)]
        n = len(shard)
        start = (step * args.chunk) % max(1, n)
        idx = (start + np.arange(args.chunk)) % max(1, n)
        return [shard[idx]]

    # N > 1 (strong scaling): every model's order is cut into units of --unit partitions, assigned
    # to ranks by LPT on the previous step's cost (sum of BaB node expansions + a fixed cost per
    # partition; a size prior before the first step), all-reduced once per step
    # --emulate-shard r/N: rank r's share of an N-rank job -- with the LPT balancer, the warmup steps
    # run EVERY unit here (the costs all ranks would all-reduce) and the timed steps rank r's units
    em_r, em_n = (int(v) for v in args.emulate_shard.split("/")) if args.emulate_shard else (0, 1)
    world_b = em_n if args.emulate_shard else info.world
    rank_b = em_r if args.emulate_shard else info.rank
    balanced = args.scope == "suite" and world_b > 1 and not args.no_balance
    U = max(1, args.unit)
    units = BL.make_units(len(models), len(order), U) if balanced else []
    # cost of a BaB node / of a partition's fixed stages (sim, prune, replay) by model: a node of
    # AC-4 (100-100) costs ~30x one of AC-8 (5-5) in the bound kernels -- weight by the network's
    # multiply-adds (plus a launch / latency floor)
    def _macs(m):
        d = [m.n_in] + m.widths
        return float(sum(d[i] * d[i + 1] for i in range(len(d) - 1)))

    # per-node constant (FAIRIFY_NODE_W_C: A/B override).  A c = 10 fit of the per-model BaB time per
    # node (narrow nets 5.6-17 ns, AC-4 51 ns) did not balance the 8 emulated ranks better than
    # c = 1: max/mean 1.040 vs 1.022, max 153.8 vs 154.0 ms (profiles/r3/ab/lpt_node_weight.md)
    node_c = float(os.environ.get("FAIRIFY_NODE_W_C", "1"))
    node_w = [node_c + _macs(m) / 256.0 for m in models]
    FIXED_COST = 64.0                      # node-equivalents per partition
    ucost = np.array([len(BL.unit_ids(order, j, U)) * FIXED_COST * node_w[k] for k, j in units], dtype=np.float64)
    assigned_cost = []

    def items_for_step(step: int):
        """[(model, item key, ids, unit indices or None)] of this rank for step ``step``."""
        if not balanced:
            return [(k, j, ids, None) for k in range(len(models)) for j, ids in enumerate(chunks_for_step(step))
                    if len(ids)]
        assign = BL.lpt_assign(ucost, world_b)
        # the loads LPT PREDICTS from the cost vector it assigned with (previous step's node counts),
        # kept with that vector: the JSON's balance fields come from one and the same prediction
        assigned_cost.append((BL.rank_loads(assign, ucost), float(ucost.max())))
        by_model = {}
        mine = assign[rank_b] if not (args.emulate_shard and step < args.warmup) else range(len(units))
        for ui in mine:
            by_model.setdefault(units[ui][0], []).append(ui)
        out = []
        for k, lst in sorted(by_model.items()):
            lst.sort(key=lambda ui: units[ui][1])
            cur, n = [], 0
            for ui in lst:
                cur.append(ui)
                n += len(BL.unit_ids(order, units[ui][1], U))
                if n >= args.chunk:
                    out.append((k, ("u", cur[0]), np.concatenate([BL.unit_ids(order, units[x][1], U) for x in cur]), cur))
                    cur, n = [], 0
            if cur:
                out.append((k, ("u", cur[0]), np.concatenate([BL.unit_ids(order, units[x][1], U) for x in cur]), cur))
        return out

    conc = args.concurrency or (BL.host_threads(8, 2) if info.device.type == "cuda" else 1)
    cfg.smt_workers = BL.host_threads(12, 1)

    timer = StageTimer(info.device, sync=args.profile)

    # Work items = (model, chunk of its shard), largest models first; a pool of host threads,
    # each driving its own HIP stream (the native BaB loop releases the GIL), so one chunk's
    # host phases overlap other chunks' kernels and big models no longer serialise the tail.
    tls = threading.local()

    def thread_stream(high: bool = False):
        """This thread's HIP stream; ``high``: its high-priority twin (the critical-path items)."""
        if info.device.type != "cuda":
            return contextlib.nullcontext()
        if getattr(tls, "stream", None) is None:
            tls.stream = torch.cuda.Stream(info.device)
            lo_pri, hi_pri = torch.cuda.Stream.priority_range()
            tls.stream_hi = torch.cuda.Stream(info.device, priority=hi_pri) if hi_pri != lo_pri else tls.stream
        return torch.cuda.stream(tls.stream_hi if high else tls.stream)

    # the heaviest items of a step (longest previous wall time) run on high-priority streams:
    # with fewer items than host threads per GPU (small shards) their dependent chain of BaB
    # levels is the step's critical path, the light items fill the gaps (0 = off)
    n_hi = args.priority_items

    pool = ThreadPoolExecutor(max_workers=conc) if conc > 1 else None

    # measured wall time per (model, chunk slot) from the previous step: the next step schedules
    # the longest items first (LPT), so the slowest model's chain starts at t=0 instead of after
    # a wave of cheap items (prior before any measurement: model size)
    item_cost = {}
    ITEM_LOG = os.environ.get("FAIRIFY_BENCH_ITEMS") == "1"   # per-item start / duration on stderr
    if ITEM_LOG:   # Python garbage collections (they hold the GIL: every host thread stalls)
        import gc

        _gc_t = {}

        def _gc_cb(phase, info_):
            if phase == "start":
                _gc_t["t"] = time.time()
            elif info_.get("generation", 0) >= 1:
                print(f"[gc] step {step_no[0]} gen {info_['generation']} at {_gc_t['t'] - step_t0[0]:.3f}s "
                      f"took {1e3 * (time.time() - _gc_t['t']):.2f} ms collected {info_.get('collected')}",
                      file=sys.stderr, flush=True)

        gc.callbacks.append(_gc_cb)
    step_no, step_t0 = [0], [time.time()]
    # counters: attempted, decided, sat, unsat, unsat_heuristic, sat per stage, unsat per stage
    # (STAGES order)
    NC = 5 + 2 * len(STAGES)
    # per model: attempted, unknown (no verdict), sound-unknown (no SOUND verdict), node expansions per
    # stage (engine/pipeline.py:STAGE_NODE_COLS)
    from fairify_amd.engine.pipeline import STAGE_NODE_COLS

    NPM = 3 + len(STAGE_NODE_COLS)
    pm_tot = np.zeros((len(models), NPM))

    def one_item(k: int, j, ids: np.ndarray, uis=None, high: bool = False):
        m, be = models[k], backends[k]
        t_item = time.time()
        with thread_stream(high):
            recs = verify_chunk(be, m, q, grid, ids, cfg, timer=timer)
            if info.device.type == "cuda":
                torch.cuda.current_stream(info.device).synchronize()
        item_cost[(k, j)] = time.time() - t_item
        if ITEM_LOG:
            print(f"[item] step {step_no[0]} {models[k].name} chunk {j} n={len(ids)} start "
                  f"{t_item - step_t0[0]:.3f}s took {item_cost[(k, j)]:.3f}s", file=sys.stderr, flush=True)
        v, st = recs.cols["verdict"], recs.cols["stage"]
        sat, uns = v == "sat", v == "unsat"
        out = np.zeros(NC, dtype=np.float64)
        out[:5] = [len(recs), sat.sum() + uns.sum(), sat.sum(), uns.sum(), (uns & (st == "heuristic")).sum()]
        for i, name in enumerate(STAGES):
            out[5 + i] = (sat & (st == name)).sum()
            out[5 + len(STAGES) + i] = (uns & (st == name)).sum()
        pm = np.zeros(NPM)
        sound = (sat & (st != "heuristic")) | (uns & ~np.isin(st, UNSOUND_UNSAT))
        pm[:3] = [len(recs), (~(sat | uns)).sum(), (~sound).sum()]
        sn = recs.cols.get("stage_nodes")
        if sn is not None:
            pm[3:] = sn.sum(axis=0)
        costs = {}
        if uis is not None:      # per-unit cost of the next step's LPT: node expansions + fixed cost
            nodes = recs.cols["nodes"].astype(np.float64)
            o = 0
            for ui in uis:
                nu = len(BL.unit_ids(order, units[ui][1], U))
                costs[ui] = node_w[k] * (float(nodes[o:o + nu].sum()) + FIXED_COST * nu)
                o += nu
        return out, costs, (k, pm)

    def run_step(step: int, timed: bool = False):
        step_no[0], step_t0[0] = step, time.time()
        items = items_for_step(step)
        items.sort(key=lambda it: (-item_cost.get((it[0], it[1]), 0.0), -models[it[0]].n_neurons))
        res = []
        if pool is None:
            res = [one_item(k, j, ids, uis) for k, j, ids, uis in items]
        else:
            res = [f.result() for f in [pool.submit(one_item, k, j, ids, uis, i < n_hi)
                                        for i, (k, j, ids, uis) in enumerate(items)]]
        if timed:
            for _, _, (k, pm) in res:
                pm_tot[k] += pm
        if balanced:
            local = np.zeros(len(units))
            for _, costs, _ in res:
                for ui, cval in costs.items():
                    local[ui] = cval
            if args.emulate_shard:
                if step < args.warmup:
                    ucost[:] = local                             # every unit ran here
            else:
                ucost[:] = D.all_reduce_sum(info, local)         # every unit ran on exactly one rank
        return sum((o for o, _, _ in res), np.zeros(NC))

    sync = (lambda: torch.cuda.synchronize(info.device)) if info.device.type == "cuda" else (lambda: None)

    def marker(tag: int):
        # fa_trace_marker_kernel brackets the timed steps in a rocprofv3 kernel trace
        # (tools/trace_busy.py --window: GPU busy fraction of exactly the timed region)
        if info.device.type == "cuda":
            from fairify_amd.ops import hip as H

            H.trace_marker(info.device, tag)

    for w in range(args.warmup):
        run_step(w)
    sync()
    from fairify_amd.utils import heap

    if os.environ.get("FAIRIFY_GC_FREEZE", "1") != "0":
        heap.freeze()     # no generation-2 pass over the setup heap inside the timed steps
    D.barrier(info)
    sync()
    mem0 = _native_mem()
    marker(1)
    t0 = time.time()
    tot = np.zeros(NC)
    for s in range(args.steps):
        tot += run_step(args.warmup + s, timed=True)
    sync()
    marker(2)
    t_local = time.time() - t0          # this rank's own work, before waiting for the others
    D.barrier(info)
    sync()
    dt = time.time() - t0
    dt_max = D.all_reduce_max(info, dt)
    rank_ms = D.all_gather_floats(info, 1000.0 * t_local / max(1, args.steps))
    tot = D.all_reduce_sum(info, tot)
    pm_all = D.all_reduce_sum(info, pm_tot.reshape(-1)).reshape(pm_tot.shape) / max(1, args.steps)
    att, dec, sat, uns, uns_h = tot[:5].tolist()
    sat_stage = {name: int(tot[5 + i]) for i, name in enumerate(STAGES)}
    unsat_stage = {name: int(tot[5 + len(STAGES) + i]) for i, name in enumerate(STAGES)}
    # sound = SAT confirmed on the original network + UNSAT from rigorous proofs (heuristic-retry
    # UNSAT and a trusted MILP's floating-point UNSAT excluded; a heuristic SAT that does not flip
    # the original network excluded)
    uns_unsound = sum(unsat_stage[k] for k in UNSOUND_UNSAT)
    dec_sound = dec - uns_unsound - sat_stage["heuristic"]
    value = dec_sound / dt_max if dt_max > 0 else 0.0
    per_step = att / max(1, args.steps)
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "soundly decided partitions/s (confirmed SAT + proved UNSAT, whole job)",
        "n_gpus": info.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * dt_max / max(1, args.steps), 3),
        "higher_is_better": True,
        "scaling": "strong" if args.scope == "suite" else "weak",
        "vs_baseline": round(value / BASELINE_DECIDED_PER_S, 1),
        "dtype": "fp32",
        "data": f"synthetic: reference src/AC integer domain, {args.weights}-init AC-1..12 weights",
        "config": {"model": f"AC suite ({','.join(names)})", "global_batch": int(per_step), "seq_len": None,
                   "parallelism": f"dp{info.world}", "preset": args.preset, "grid_per_model": len(order),
                   "sim_size": cfg.sim_size, "node_budget": cfg.node_budget,
                   "escalate_budget": cfg.escalate_budget, "escalate_max_open": cfg.escalate_max_open,
                   "heuristic_node_budget": cfg.heuristic_node_budget, "relu_budget": cfg.relu_budget,
                   "relu_max_width": cfg.relu_max_width, "relu_escalate_cap": cfg.relu_escalate_cap,
                   "beta_budget": cfg.beta_budget, "anytime_beta": cfg.anytime_beta,
                   "escalate_probation": [list(st) for st in cfg.escalate_probation],
                   "stages": [list(st) for st in cfg.escalate_stages], "heuristic": cfg.heuristic,
                   "batch_nodes": cfg.batch_nodes,
                   "chunk": args.chunk, "concurrency": conc, "priority_items": args.priority_items},
        "decided_per_s_all": round(dec / dt_max, 3) if dt_max > 0 else 0.0,
        "pct_verified": round(100.0 * dec / max(1.0, att), 3),
        "pct_verified_sound": round(100.0 * dec_sound / max(1.0, att), 3),
        "partitions_per_s": round(att / dt_max, 3) if dt_max > 0 else 0.0,
        "sat": int(sat), "unsat": int(uns), "unknown": int(att - dec),
        "unsat_sound": int(uns - uns_unsound), "unsat_heuristic": int(uns_h), "sat_by_stage": sat_stage,
        "unsat_by_stage": unsat_stage,
        "dist": {"world": info.world, "backend": backend_name,
                 "rank_ms_per_step": [round(x, 1) for x in rank_ms],
                 "skew_ms": round(max(rank_ms) - min(rank_ms), 1) if rank_ms else 0.0,
                 "balance": ("lpt" if balanced else "strided"), "unit": U if balanced else None,
                 # predicted per-rank loads of the last timed step's assignment (node-count costs of
                 # the step before it, parallel/balance.py), its makespan over the ideal even split,
                 # and LPT's guarantee for the same cost vector, (mean + largest unit) / mean
                 "predicted_rank_cost": [round(float(c), 1) for c in assigned_cost[-1][0]] if assigned_cost else None,
                 "predicted_cost_ratio": (round(float(max(assigned_cost[-1][0]) /
                                                      max(1e-9, np.mean(assigned_cost[-1][0]))), 4)
                                          if assigned_cost else None),
                 "predicted_cost_bound": (round(float(1.0 + assigned_cost[-1][1] /
                                                      max(1e-9, np.mean(assigned_cost[-1][0]))), 4)
                                          if assigned_cost else None),
                 "host_cpus": len(cpus), "host_threads": conc,
                 # native runtimes' caching allocator (csrc/devmem.h) over the timed steps:
                 # driver-level frees stall every host thread; steady state = 0
                 "native_mem": _mem_delta(mem0, _native_mem())},
        "baseline": {"decided_per_s": round(BASELINE_DECIDED_PER_S, 5), "pct_verified_of_attempted": 89.0,
                     "coverage_of_grid_pct": 0.29},
        # vs_baseline divides this random-init rate by the reference's TRAINED-weight Table-V rate: a
        # cross-regime ratio.  The trained-weight comparison at equal budgets is its own run
        # (tools/baseline_configs.py --group tablev; profiles/r6/baseline_configs.md).
        "vs_baseline_note": "cross-regime: random-init AC suite (this run) / trained-weight Table V AC-sex "
                            "aggregate (553 decided in 22 144 s); trained Table V at one HEAD: "
                            "profiles/r6/baseline_configs.md",
        # per model and per timed step: attempted, unknown, sound-unknown (no sound verdict) and node
        # expansions per stage
        "per_model": {m.name: {"attempted": int(round(pm_all[k, 0])), "unknown": round(float(pm_all[k, 1]), 1),
                               "unknown_sound": round(float(pm_all[k, 2]), 1),
                               "nodes": {c: int(round(pm_all[k, 3 + i])) for i, c in enumerate(STAGE_NODE_COLS)}}
                      for k, m in enumerate(models)},
    }
    if args.budget_pass > 0:
        # per-model wall budget B: every (model, chunk) item gets the chunk's share of B for its
        # anytime phase; items of all models run concurrently on the host streams, so the pass
        # takes about B plus the fixed-schedule time of one step
        from dataclasses import replace as _replace

        chunks = chunks_for_step(0)
        n_shard = max(1, sum(len(c) for c in chunks))
        bcfg = {k: _replace(cfg, smt_backend="auto", anytime_seconds=args.budget_pass * len(c) / n_shard)
                for k, c in enumerate(chunks)}
        NB = 2 + len(STAGES) + 2 + len(STAGES)

        def budget_item(k: int, j: int, ids: np.ndarray):
            with thread_stream():
                recs = verify_chunk(backends[k], models[k], q, grid, ids, bcfg[j], timer=timer)
                if info.device.type == "cuda":
                    torch.cuda.current_stream(info.device).synchronize()
            v, st = recs.cols["verdict"], recs.cols["stage"]
            sat, uns = v == "sat", v == "unsat"
            o = np.zeros(NB)
            o[0], o[1] = len(recs), sat.sum() + uns.sum()
            for i, name in enumerate(STAGES):
                o[2 + i] = (uns & (st == name)).sum()
            o[2 + len(STAGES)] = sat.sum()
            o[3 + len(STAGES)] = uns.sum()
            for i, name in enumerate(STAGES):
                o[4 + len(STAGES) + i] = (sat & (st == name)).sum()
            return o

        D.barrier(info)
        tb = time.time()
        items = [(k, j, ids) for k in range(len(models)) for j, ids in enumerate(chunks) if len(ids)]
        items.sort(key=lambda it: -models[it[0]].n_neurons)
        if pool is None:
            btot = sum(budget_item(*it) for it in items)
        else:
            btot = sum(f.result() for f in [pool.submit(budget_item, *it) for it in items])
        sync()
        D.barrier(info)
        bwall = D.all_reduce_max(info, time.time() - tb)
        btot = D.all_reduce_sum(info, np.asarray(btot, dtype=np.float64))
        out["pct_verified_at_budget"] = round(100.0 * btot[1] / max(1.0, btot[0]), 3)
        b_uns = {name: int(btot[2 + i]) for i, name in enumerate(STAGES)}
        b_sat = {name: int(btot[4 + len(STAGES) + i]) for i, name in enumerate(STAGES)}
        b_sound = btot[1] - sum(b_uns[k] for k in UNSOUND_UNSAT) - b_sat["heuristic"]
        out["pct_verified_at_budget_sound"] = round(100.0 * b_sound / max(1.0, btot[0]), 3)
        out["budget_pass"] = {
            "seconds_per_model": args.budget_pass, "wall_s": round(bwall, 2), "attempted": int(btot[0]),
            "decided": int(btot[1]), "sat": int(btot[2 + len(STAGES)]), "unsat": int(btot[3 + len(STAGES)]),
            "unsat_by_stage": {name: int(btot[2 + i]) for i, name in enumerate(STAGES) if btot[2 + i]},
            "sat_by_stage": {k: v for k, v in b_sat.items() if v},
            "note": "untimed; anytime mode: falsifier rounds, input-split BaB budgets x4 per round, "
                    "ReLU-phase BaB, verified-LP rounds (stage 'lp': UNSAT from certified weak-duality "
                    "bounds; --lp-budget 0 --trust-milp: HiGHS MILP instead), heuristic retry last; "
                    "pct_verified_at_budget_sound excludes heuristic (and trusted-MILP) verdicts"}
    if args.profile and info.is_main:
        print(timer.report(), file=sys.stderr, flush=True)
    if info.is_main:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if pool is not None:
        pool.shutdown(wait=True)
    D.destroy(info)


if __name__ == "__main__":
    main()
