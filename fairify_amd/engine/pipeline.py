"""Per-model verification pipeline over a stream of partition chunks.

Re-design of the per-partition loop of the reference drivers (``src/GC/Verify-GC.py:106-315``):
sound prune -> SMT query -> heuristic prune + re-query on ``unknown`` -> counterexample replay
-> one CSV row per partition -> hard timeout.  Here a *chunk* of partitions (thousands) goes
through each stage at once on the device:

  decode ids -> simulate/profile/falsify (K3+K8) -> IBP bounds (K2, B-compression) ->
  symbolic bounds (K4, S-compression) -> branch-and-bound (K9) -> [heuristic masks (K5) +
  BaB on the masked nets for UNKNOWN partitions] -> replay (K7) -> records.

Per-partition timings are the chunk's stage times apportioned by each partition's share of
the work (BaB node expansions), so the 24 CSV columns keep their meaning.
"""
from __future__ import annotations

import os
import sys
import time
from dataclasses import dataclass, field, replace
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..models.mlp import MLP
from ..ops.backend import Backend
from ..partition import Grid
from ..spec import ResolvedQuery
from . import exact
from . import prune as P_
from .bab import SAT, UNKNOWN, UNSAT, RUNNING, VERDICT_NAMES, BaBConfig, BaBSolver, _pa_table, pa_groups
from .falsify import residual_falsify
from .sim import simulate
from ..utils import faults
from ..utils.timer import StageTimer


def _host_workers(cap: int) -> int:
    from ..parallel.balance import host_threads

    return host_threads(cap, 1)


@dataclass
class VerifyConfig:
    sim_size: int = 1000                 # reference sim_size (src/AC/Verify-AC.py:115)
    seed: int = 0
    chunk: int = 4096                    # partitions per device batch
    soft_timeout: float = 100.0          # seconds (caps one chunk's BaB wall time)
    hard_timeout: float = 30 * 60.0      # seconds per model (checked after each chunk)
    node_budget: int = 4096              # BaB expansions per partition
    escalate_budget: int = 0             # second sound BaB pass on the residue with this node
                                         # budget (0 = off); runs after the residual falsifier
    escalate_max_open: int = 0           # only escalate partitions that left at most this many
                                         # open nodes in the first pass (0 = all; native BaB only)
    escalate_stages: Tuple[Tuple[int, int], ...] = ()
    # inline escalation steps between node_budget and escalate_budget: (budget, max frontier) --
    # a partition continues past each step's budget only if its open frontier at that level is at
    # most the limit (the first step uses escalate_max_open)
    escalate_probation: Tuple[Tuple[int, int], ...] = ()
    inline_escalate: bool = True         # native BaB: run the escalate_budget stage inside the first
                                         # pass (escalate_max_open then bounds the frontier size)
                                         # further (budget, max_open) passes after the escalated one,
                                         # each on the residue the previous pass left
    batch_nodes: int = 65536             # BaB nodes per sub-batch launch
    heuristic: bool = True               # reference behaviour: heuristic retry on unknown
    heuristic_p: float = 5.0             # HEURISTIC_PRUNE_THRESHOLD
    heuristic_node_budget: int = 4096
    bisect_pairs: int = 16
    bisect_steps: int = 0                # boundary walk in the sim stage; 0 = off (the residual
                                         # falsifier finds the same witnesses: A/B 87.32 vs 87.32 %)
    sound_prune_stats: bool = True       # compute B/S compression (reference parity columns)
    residual_samples: int = 2048         # residual falsifier on BaB-UNKNOWN partitions (0 = off)
    residual_starts: int = 16            # local-search starts per partition
    residual_iters: int = 12             # coordinate-ascent rounds
    smt_backend: str = "auto"            # exact host solver on the BaB residue: auto (Z3 if installed,
                                         # else the HiGHS MILP back-end) | z3py | z3bin | milp | none
    # host solver processes (LP / MILP / SMT): the rank's CPUs, at most 15 (a one-GPU share of 16
    # CPUs less the GPU driver thread; trained AC-7 at 120 s: 12 workers 74.5 / 85.2 % sound,
    # 15 workers 78.3 / 87.8 %); FAIRIFY_SMT_WORKERS overrides
    smt_workers: int = field(default_factory=lambda: int(os.environ.get("FAIRIFY_SMT_WORKERS", "0"))
                             or _host_workers(15))
                                         # host solver threads: this rank's CPUs (its node slice when
                                         # several ranks share a node, parallel/balance.py), at most 12
    smt_timeout: Optional[float] = None  # per query; defaults to soft_timeout
    smt_fork_params: bool = False        # Z3 seed/restart/phase options of the fork's drivers
    # anytime mode: after the fixed passes, keep growing the node budget (x anytime_growth per
    # round) and the residual falsifier's sample count on the sound-UNKNOWN residue until it is
    # empty or this chunk's share of the model's wall budget is spent (the reference spends up to
    # its hard timeout per model, src/AC/Verify-AC.py:318-320).  0 = off.
    anytime_seconds: float = 0.0
    pruned_metrics: bool = False         # Pruned-F1 counts for every partition (the experiment
                                         # drivers' per-partition metrics CSV)
    anytime_growth: int = 4
    anytime_max_budget: int = 1 << 22
    anytime_pool: int = 1 << 24          # live BaB nodes per group: group size = pool / budget
    anytime_max_samples: int = 16384
    anytime_milp_seconds: float = 1.0    # first MILP round's per-partition limit (x growth per round)
    # a GPU stage (input-split / ReLU-phase BaB) whose anytime round decides less than this fraction
    # of the partitions it attempted is not run in later rounds: its next budget (x growth) would
    # spend the remaining time where it does not converge (trained AC-7: 1.6 G input-split nodes in
    # 110 s for 424 proofs) -- the other stages get it
    anytime_min_yield: float = 0.01
    # the first anytime round's verified-LP node budget is lp_budget / this (x growth per round);
    # 0 = by the PA table: a binary PA (2 ordered pairs) starts at 1/4 -- many cheap attempts first
    # (trained AC-7/sex at 120 s: 78.8 % vs 72.8 % at the full budget) --, a multi-valued PA at the
    # full budget, where the per-value sign tests need it (AC-7/race: 99.8 % vs 87.8 %)
    anytime_lp_div: int = int(os.environ.get("FAIRIFY_ANYTIME_LP_DIV", "0"))
    relu_budget: int = 2048              # ReLU-phase BaB (stage "relu", engine/relu_bab.py) on the
                                         # input-split residue: nodes per partition (0 = off)
    relu_max_width: int = 16             # ... only for networks whose hidden layers are at most this
                                         # wide (the narrow zero-bias shapes it closes; on the wide AC
                                         # shapes it spends its budget without deciding: tools/diag_relu.py)
    relu_escalate_cap: int = 0           # networks the relu stage runs on: cap the input-split
                                         # escalation budget at this (their residue goes to the cheaper
                                         # relu stage instead of deep input splitting; 0 = no cap)
    relu_first: bool = True              # relu-covered networks: the (capped) input-split escalation
                                         # runs AFTER the relu stage, on what it left, instead of inline
                                         # in the first pass -- most of their escalated partitions are
                                         # zero-logit boxes the relu stage closes in a few nodes
                                         # (profiles/r3/shard/diag_models_bench_config.jsonl: 38 % of a
                                         # bench step's nodes were AC-8 / AC-12 escalation spent on
                                         # partitions the relu stage then decided)
    beta_budget: int = int(os.environ.get("FAIRIFY_BETA_BUDGET", "128"))
                                         # beta-CROWN phase-split BaB (stage "beta", engine/beta_bab.py)
                                         # on the residue: nodes per partition (0 = off); the trained
                                         # AC-7 residue closes in 10-60 nodes, the random-init bench
                                         # residue mostly does not (512 nodes: +3.4 s per step for 147
                                         # verdicts, gpurun_out/s5_c); 128 with probe 8 over 64 with
                                         # probe 4: targeted/AC AC-7 97.29 -> 98.30 % for +7 % time
                                         # (profiles/r5/s5_u/); the anytime rounds grow it x
                                         # anytime_growth per round
    anytime_beta: int = 64               # anytime rounds: beta BaB nodes per partition of the first round
                                         # (x anytime_growth per round; 0 = off), independent of the
                                         # fixed-pass beta_budget
    # fixed pass: a partition gives up once it has expanded 2 x this many nodes per pair tree with none
    # of its trees closed (0 = never)
    beta_probe_levels: int = int(os.environ.get("FAIRIFY_BETA_PROBE", "8"))
    beta_min_width: int = 17             # ... on networks whose widest hidden layer is at least this
                                         # (the narrower ones go to the relu stage, whose exact-zero
                                         # concretisation their zero logits need)
    beta_max_width: int = 256            # ... and at most this (fixed pass only).  BM-4's 150-wide layer ran in
                                         # round 5 with its weights staged in LDS (2 waves per CU) and decided
                                         # 1.5 % of its residue; with the weights read from L2 (7 waves per
                                         # CU) and primal-gap branching relaxed/BM BM-4 goes 11 118 -> 8 532
                                         # UNKNOWN (98.89 -> 99.15 %) for 49.8 -> 68.3 s (profiles/r6/); a
                                         # static rule, so verdicts stay independent of the sharding
    beta_branch: str = os.environ.get("FAIRIFY_BETA_BRANCH", "auto")
                                         # BetaConfig.branch: "pgap" = the verified LP's primal-gap rule
                                         # at the averaged primal iterate (relaxed/BM BM-8 residue: 33 vs
                                         # 5 of 200 decided at 1 024 nodes, profiles/r6/), "kernel" =
                                         # |lambda| x gap at the vertex x* (round 5); "auto": pgap with
                                         # beta_iters steps for a binary PA (2 ordered pairs), kernel with
                                         # 64 for a multi-valued one -- measured per query at the fixed
                                         # pass's budget: relaxed/BM BM-8 17 866 vs 22 785 UNKNOWN (pgap /
                                         # kernel), stress/AC AC-7 4 466 vs 4 668, but relaxed/AC AC-7
                                         # (race, 20 pairs) 1 840 vs 1 755 at 27.3 vs 18.9 s (profiles/r6/)
    beta_iters: int = int(os.environ.get("FAIRIFY_BETA_ITERS", "128"))
                                         # optimisation steps per child node (root: x 3); 128 over 64:
                                         # 48 vs 33 of 200 at 1 024 nodes (a converged dual gives the
                                         # primal average its meaning)
    beta_lookahead: int = 8              # filtered look-ahead candidates per score list
    beta_decay: float = float(os.environ.get("FAIRIFY_BETA_DECAY", "0.98"))
                                         # step-size decay per optimisation step (BetaConfig.decay)
    beta_feas_iters: int = int(os.environ.get("FAIRIFY_BETA_FEAS", "0"))
                                         # infeasibility pass steps on open children (BetaConfig.feas_iters)
                                         # in the fixed pass: off -- at its 128-node budget with the probe
                                         # it decided nothing more (relaxed/BM BM-8 17 866 vs 18 234 UNKNOWN,
                                         # profiles/r6/); the anytime rounds (growing budgets) run 64 steps
    beta_escalate_cap: int = int(os.environ.get("FAIRIFY_BETA_ESC_CAP", "0"))
                                         # networks the beta fixed pass runs on: cap the input-split
                                         # escalation budget at this (their residue goes to beta instead
                                         # of deep input splitting; 0 = no cap)
    lp_budget: int = 4096                # verified-LP branch-and-bound (stage "lp", smt/lpbab.py) in
                                         # place of the untrusted MILP: LP nodes per partition (x growth
                                         # per anytime round); 0 = the round-2 MILP stage
    trust_milp: bool = False             # HiGHS MILP UNSAT rests on a floating-point dual bound: by
                                         # default it is recorded (stage "milp") but the partition
                                         # stays UNKNOWN for the rigorous stages; True = round-2
                                         # behaviour (UNSAT, stage "milp", excluded from sound counts)
    keep_masks: bool = False             # K6: keep every partition's final dead-neuron mask (sound
                                         # prune, or the heuristic mask of a retried partition) as a
                                         # packed bitset (core["mask_bits"], ceil(N/8) B) for the
                                         # rank-0 gather, dedup and pruned-subnet export

    def __post_init__(self):
        # the rank-0 wire records (parallel/wire.py) carry the agree / tp / fp counts of the
        # simulation points as uint16: reject a sample count they cannot hold here, before any
        # rank has done GPU work (a late OverflowError would leave the other ranks in the gather)
        if not 0 < int(self.sim_size) <= 65535:
            raise ValueError(f"sim_size must be in 1..65535 (got {self.sim_size})")


@dataclass
class PartitionRecord:
    partition_id: int                    # 1-based position in processing order (reference)
    grid_id: int
    verdict: str
    h_attempt: int = 0
    h_success: int = 0
    b_comp: float = 0.0
    s_comp: float = 0.0
    st_comp: float = 0.0
    h_comp: float = 0.0
    t_comp: float = 0.0
    sv_time: float = 0.0
    s_time: float = 0.0
    hv_time: float = 0.0
    h_time: float = 0.0
    total_time: float = 0.0
    c_check: int = 0
    v_accurate: int = 0
    orig_acc: Optional[float] = None
    pruned_acc: float = 1.0
    c1: Optional[np.ndarray] = None
    c2: Optional[np.ndarray] = None
    nodes: int = 0
    stage: str = ""                      # which stage decided: sim / bab / heuristic


@dataclass
class ModelRun:
    model: str
    records: List[PartitionRecord] = field(default_factory=list)
    attempted: int = 0
    wall: float = 0.0
    stopped_by_hard_timeout: bool = False

    def counts(self) -> Dict[str, int]:
        c = {"sat": 0, "unsat": 0, "unknown": 0}
        for r in self.records:
            c[r.verdict] += 1
        return c


class _LazyMasked:
    """Per-partition heuristically pruned networks, materialised only when a SAT candidate of
    that partition needs exact confirmation."""

    def __init__(self, mlp: MLP, masks: List[np.ndarray], widths):
        self.mlp, self.masks, self.sls = mlp, masks, P_.layer_slices(widths)
        self.cache: Dict[int, MLP] = {}

    def __getitem__(self, k: int) -> MLP:
        if k not in self.cache:
            self.cache[k] = self.mlp.masked([self.masks[k][s] for s in self.sls])
        return self.cache[k]

    def __len__(self) -> int:
        return len(self.masks)


_HOST_SMT: Dict[tuple, object] = {}
_VERBOSE_ANYTIME = os.environ.get("FAIRIFY_VERBOSE_ANYTIME") == "1"


def _host_smt(cfg: VerifyConfig):
    """Host SMT pool for the residue (cached per configuration; inactive without a back-end)."""
    from ..smt.host import HostSMT

    key = (cfg.smt_backend, cfg.smt_workers, cfg.smt_timeout or cfg.soft_timeout, cfg.smt_fork_params)
    if key not in _HOST_SMT:
        _HOST_SMT[key] = HostSMT(cfg.smt_backend, cfg.smt_workers, key[2], cfg.smt_fork_params)
    return _HOST_SMT[key]


def _amortize(total: float, work: np.ndarray) -> np.ndarray:
    w = work.astype(np.float64) + 1.0
    return total * w / w.sum()


def _milp_round(be, mlp, q, unk, lo_np, hi_np, values_np, pairs_np, limit, workers, status, stage, cex_x, cex_xp,
                deadline=None, trust: bool = False):
    """HiGHS MILP on the partitions ``unk`` (per-partition time limit ``limit``, nothing starts
    after ``deadline``); exactly confirmed SAT verdicts are written into the stage arrays.  An
    UNSAT answer (floating-point dual bound) is only recorded as stage ``milp`` on a partition that
    stays UNKNOWN, unless ``trust`` (then it is an UNSAT verdict of stage ``milp``)."""
    from ..smt import milp

    futs = milp.submit(be, mlp, q, lo_np[unk], hi_np[unk], values_np, pairs_np, limit, workers=workers,
                       deadline=deadline)
    cand_k, cand_x, cand_xp = [], [], []
    t_note = time.time()
    for i, (k, f) in enumerate(zip(unk, futs)):
        verdict, pair = f.result()
        if _VERBOSE_ANYTIME and time.time() - t_note > 30.0:
            t_note = time.time()
            print(f"[milp] {mlp.name}: {i + 1}/{len(unk)} partitions, limit {limit:.1f}s", flush=True)
        if verdict == "unsat":
            stage[k] = "milp"
            if trust:
                status[k] = UNSAT
        elif verdict == "sat" and pair is not None:
            cand_k.append(k)
            cand_x.append(pair[0])
            cand_xp.append(pair[1])
    if cand_k:
        ck_ = np.asarray(cand_k)
        X, XP = np.asarray(cand_x, dtype=np.int64), np.asarray(cand_xp, dtype=np.int64)
        ok = exact.check_pair_constraints(X, XP, lo_np[ck_], hi_np[ck_], q.pa_idx, q.ra_idx, q.tau)
        viol = exact.is_violation(mlp, X, XP) & ok
        hit = ck_[viol]
        status[hit] = SAT
        cex_x[hit], cex_xp[hit] = X[viol], XP[viol]
        stage[hit] = "milp"


def _beta_round(be, q, mlp, unk, lo_np, hi_np, budget, time_budget, batch_nodes, status, stage, cex_x, cex_xp, nodes,
                tm=None, probe_levels: int = 0, cfg=None, anytime: bool = False):
    """beta-CROWN BaB (engine/beta_bab.py) on the partitions ``unk``: decided verdicts (sound SAT /
    UNSAT) written into the stage arrays; returns how many it decided.  ``probe_levels``: a partition
    gives up once it has expanded 2 x that many nodes per pair tree with none of its trees closed
    (BetaConfig)."""
    from .beta_bab import BetaBaBSolver, BetaConfig

    kw = {}
    if cfg is not None:
        branch, iters = cfg.beta_branch, cfg.beta_iters
        if branch == "auto":
            from .bab import _pa_table

            _, pairs = _pa_table(q, lo_np[unk[:1]], hi_np[unk[:1]])
            branch, iters = ("pgap", cfg.beta_iters) if pairs.shape[0] <= 2 else ("kernel", 64)
        kw = dict(branch=branch, iters=iters, root_iters=max(200, 3 * iters),
                  lookahead=cfg.beta_lookahead, decay=cfg.beta_decay,
                  feas_iters=max(cfg.beta_feas_iters, 64) if anytime else cfg.beta_feas_iters)
    bs = BetaBaBSolver(be, q, BetaConfig(node_budget=budget, batch_nodes=min(batch_nodes, 32768),
                                         time_budget=time_budget, probe_levels=probe_levels, **kw),
                       **({"timer": tm} if tm is not None else {}))
    t0 = time.time()
    br = bs.solve(lo_np[unk], hi_np[unk], mlp)
    dec = np.isin(br.status, (SAT, UNSAT))
    if os.environ.get("FAIRIFY_BETA_LOG"):
        print(f"[beta] {unk.size} partitions, budget {budget}: decided {int(dec.sum())} in "
              f"{time.time() - t0:.2f} s, {bs.stats}", file=sys.stderr, flush=True)
    hit = unk[dec]
    status[hit] = br.status[dec]
    stage[hit] = "beta"
    sb = br.status == SAT
    cex_x[unk[sb]] = br.cex_x[sb]
    cex_xp[unk[sb]] = br.cex_xp[sb]
    nodes[unk] += br.nodes
    return int(dec.sum())


def _lp_round(be, mlp, q, unk, lo_np, hi_np, values_np, pairs_np, budget, limit, workers, status, stage, cex_x,
              cex_xp, deadline=None):
    """Verified-LP branch-and-bound (smt/lpbab.py) on the partitions ``unk``: HiGHS solves, a
    rigorous weak-duality bound from its multipliers closes nodes, lattice points and LP optima
    are checked exactly.  UNSAT and SAT verdicts are both sound (stage ``lp``)."""
    pending = _lp_submit(be, mlp, q, unk, lo_np, hi_np, values_np, pairs_np, budget, limit, workers, deadline)
    _lp_collect(mlp, pending, budget, status, stage, cex_x, cex_xp)


def _lp_submit(be, mlp, q, unk, lo_np, hi_np, values_np, pairs_np, budget, limit, workers, deadline=None):
    """Start the verified-LP searches of ``unk`` in the worker processes; returns [(k, future)]."""
    from ..smt import lpbab

    futs = lpbab.submit(be, mlp, q, lo_np[unk], hi_np[unk], values_np, pairs_np, budget, limit, workers=workers,
                        deadline=deadline)
    return list(zip(unk, futs))


def _lp_collect(mlp, pending, budget, status, stage, cex_x, cex_xp):
    """Wait for the LP searches of :func:`_lp_submit`; a partition another stage decided meanwhile
    keeps that verdict (both are sound)."""
    t_note = time.time()
    # searches of partitions another stage decided meanwhile: not started ones are dropped, so the
    # shared worker pool is not kept busy for nothing (running ones finish and are ignored)
    for k, f in pending:
        if status[k] != UNKNOWN:
            f.cancel()
    for i, (k, f) in enumerate(pending):
        if f.cancelled():
            continue
        verdict, pair, _ = f.result()
        if _VERBOSE_ANYTIME and time.time() - t_note > 30.0:
            t_note = time.time()
            print(f"[lp] {mlp.name}: {i + 1}/{len(pending)} partitions, budget {budget}", flush=True)
        if status[k] != UNKNOWN:
            continue
        if verdict == "unsat":
            status[k], stage[k] = UNSAT, "lp"
        elif verdict == "sat" and pair is not None:
            status[k], stage[k] = SAT, "lp"
            cex_x[k], cex_xp[k] = pair[0], pair[1]


def _lp_available() -> bool:
    """The verified-LP stage drives HiGHS through SciPy's private ``_highspy._core`` bindings (SciPy
    >= 1.15); without them the stage is off and the MILP stage runs instead of an aborting worker."""
    try:
        from scipy.optimize._highspy import _core  # noqa: F401
    except ImportError:
        return False
    return True


def _use_lp(cfg, q) -> bool:
    from ..smt import lpbab  # noqa: F401  (SciPy present: the MILP back-end resolved)

    return cfg.lp_budget > 0 and not cfg.trust_milp and _lp_available()


def verify_chunk(be: Backend, mlp: MLP, q: ResolvedQuery, grid: Grid, ids: np.ndarray, cfg: VerifyConfig,
                 orig_acc: Optional[float] = None, time_budget: Optional[float] = None,
                 timer: Optional[StageTimer] = None) -> "ChunkRecords":
    """Decide one chunk of partitions; returns its per-partition records (no cumulative columns).

    The kernels share one table of protected-attribute assignments per launch, so a chunk whose
    partitions split the PA range differently (a PA wider than the partition size, e.g. Adult
    age with P=10) is verified as one group per distinct PA range; the records come back in
    ``ids`` order with the chunk's stage times apportioned over all of its partitions."""
    lo_np, hi_np = grid.decode(ids)
    groups = pa_groups(q, lo_np, hi_np)
    if len(groups) <= 1:
        core, seg = _verify_group(be, mlp, q, ids, lo_np, hi_np, cfg, time_budget, timer, grid=grid)
    else:
        t0 = time.time()
        core, seg = None, np.zeros(5)
        for sel in groups:
            left = None if time_budget is None else time_budget - (time.time() - t0)
            gcore, gseg = _verify_group(be, mlp, q, ids[sel], lo_np[sel], hi_np[sel], cfg, left, timer, grid=grid)
            if core is None:
                core = {k: np.zeros((len(ids),) + v.shape[1:], dtype=v.dtype) for k, v in gcore.items()}
            for k, v in gcore.items():
                core[k][sel] = v
            seg += np.asarray(gseg, dtype=np.float64)
        seg = (len(ids),) + tuple(seg[1:].tolist())
    return ChunkRecords(core, orig_acc, segments=[seg], n_neurons=mlp.n_neurons, sim_size=cfg.sim_size)


def _verify_group(be: Backend, mlp: MLP, q: ResolvedQuery, ids: np.ndarray, lo_np: np.ndarray, hi_np: np.ndarray,
                  cfg: VerifyConfig, time_budget: Optional[float], timer: Optional[StageTimer],
                  grid: Optional[Grid] = None):
    """One group of partitions sharing their protected-attribute range: (core columns, segment).

    On the GPU the device boxes are decoded from the ids by ``fa_decode_kernel`` (K1); the host
    keeps its own decode (``lo_np``/``hi_np``) for the exact confirmation of candidates."""
    tm = timer if timer is not None else StageTimer()
    t_start = time.time()
    dev = be.device
    Pn, n = lo_np.shape
    widths = mlp.widths
    Nh = int(sum(mlp.hidden))
    sync = (lambda: torch.cuda.current_stream(dev).synchronize()) if dev.type == "cuda" else (lambda: None)

    values_np, pairs_np = _pa_table(q, lo_np, hi_np)
    values = torch.from_numpy(values_np).to(dev)
    pairs = torch.from_numpy(pairs_np).to(dev)
    pids = torch.from_numpy(ids).to(dev)
    if be.hip and grid is not None:
        from ..ops import hip as H

        lo, hi = H.decode(grid, pids)
    else:
        lo = torch.from_numpy(lo_np).to(dev, torch.float32)
        hi = torch.from_numpy(hi_np).to(dev, torch.float32)

    # ---------------- stage 1: simulation (profile + falsify)
    t0 = time.time()
    with tm("sim"):
        sim = simulate(be, q, lo, hi, pids, cfg.sim_size, cfg.seed, values, pairs, cfg.bisect_pairs,
                       cfg.bisect_steps)
    # stage 2 / 4 mask algebra in HIP kernels (FAIRIFY_FUSED_PRUNE=0: the PyTorch path, for A/B tests)
    fused = be.hip and cfg.sound_prune_stats and os.environ.get("FAIRIFY_FUSED_PRUNE", "1") != "0"
    status = np.full(Pn, RUNNING, dtype=np.int8)
    cex_x = np.zeros((Pn, n), dtype=np.int64)
    cex_xp = np.zeros((Pn, n), dtype=np.int64)
    stage = np.array([""] * Pn, dtype=object)
    with tm("sim.confirm"):
        found = sim.found.cpu().numpy()
        if found.any():
            fi = np.nonzero(found)[0]
            X = sim.wit_x[fi].cpu().numpy().round().astype(np.int64)
            XP = sim.wit_xp[fi].cpu().numpy().round().astype(np.int64)
            ok = exact.check_pair_constraints(X, XP, lo_np[fi], hi_np[fi], q.pa_idx, q.ra_idx, q.tau)
            viol = exact.is_violation(mlp, X, XP) & ok
            hit = fi[viol]
            status[hit] = SAT
            cex_x[hit], cex_xp[hit] = X[viol], XP[viol]
            stage[hit] = "sim"
    sync()
    t_sim = time.time() - t0

    # ---------------- stage 2: sound pruning statistics (IBP + symbolic on the partition box)
    t0 = time.time()
    ibp_lb = ibp_ub = code = None
    if fused:
        from ..ops import hip as H

        with tm("prune.bounds"):
            ibp = be.bounds(lo, hi, mode="ibp", keep_layers=True)
            ibp_lb, ibp_ub = ibp.lay_lb_full, ibp.lay_ub_full
            sym = be.bounds(lo, hi, mode="symbolic")
            code, pcnt = H.prune_masks(be, sim.counts, ibp_ub, sym.dead_u8)
            pcnt_np = pcnt.cpu().numpy().astype(np.int64)
        b_cnt, s_cnt, st_cnt = pcnt_np[:, 0], pcnt_np[:, 1], pcnt_np[:, 2]
    else:
        cand, _ = P_.candidates_from_counts(sim.counts, cfg.sim_size)
        b_dead = torch.zeros(Pn, mlp.n_neurons, dtype=torch.bool, device=dev)
        s_dead = torch.zeros_like(b_dead)
        st_dead = torch.zeros_like(b_dead)
        s_cand = cand.clone()
        if cfg.sound_prune_stats:
            with tm("prune.bounds"):
                ibp = be.bounds(lo, hi, mode="ibp", keep_layers=True)
                ibp_lb = torch.cat(ibp.layer_lb, dim=1)
                ibp_ub = torch.cat(ibp.layer_ub, dim=1)
                b_dead, b_rem = P_.bound_dead(cand, ibp_ub[:, :Nh], widths)
                b_dead = P_.ensure_one_alive(b_dead, widths)
                sym = be.bounds(lo, hi, mode="symbolic")
                s_hid = b_rem[:, :Nh] & sym.dead
                s_dead = torch.zeros_like(b_dead)
                s_dead[:, :Nh] = s_hid
                s_cand = b_rem.clone()
                s_cand[:, :Nh] = b_rem[:, :Nh] & ~s_hid
                st_dead = P_.ensure_one_alive(P_.merge(b_dead, s_dead), widths)
        b_cnt = b_dead.sum(dim=1).cpu().numpy().astype(np.int64)
        s_cnt = s_dead.sum(dim=1).cpu().numpy().astype(np.int64)
        st_cnt = st_dead.sum(dim=1).cpu().numpy().astype(np.int64)
    sync()
    t_prune = time.time() - t0

    # ---------------- stage 3: branch and bound on the original network
    t0 = time.time()
    budget = cfg.soft_timeout if time_budget is None else min(cfg.soft_timeout, time_budget)
    from .relu_bab import supported as _relu_supported

    relu_on = cfg.relu_budget > 0 and max(mlp.hidden or [0]) <= cfg.relu_max_width and _relu_supported(q)
    from .beta_bab import supported as _beta_supported

    beta_on = (cfg.beta_budget > 0 and _beta_supported(q)
               and cfg.beta_min_width <= max(mlp.hidden or [0]) <= cfg.beta_max_width)
    esc_cap = cfg.relu_escalate_cap if relu_on else (cfg.beta_escalate_cap if beta_on else 0)
    if esc_cap > 0 and cfg.escalate_budget > esc_cap:
        # the residue of these networks goes to the relu / beta stage: stop the input-split escalation early
        cap = max(esc_cap, cfg.node_budget)
        cfg = replace(cfg, escalate_budget=cap if cap > cfg.node_budget else 0,
                      escalate_probation=tuple(st for st in cfg.escalate_probation if st[0] < cap))
    # relu_first: the escalation pass (one budget, open-frontier gate) runs after stage 3r
    esc_after_relu = relu_on and cfg.relu_first and cfg.escalate_budget > cfg.node_budget and \
        os.environ.get("FAIRIFY_RELU_FIRST", "1") != "0"
    # inline escalation (native runtime): the first escalation stage runs inside the first pass --
    # partitions that reach node_budget with a small frontier continue instead of restarting from
    # the root in a second solve (FAIRIFY_INLINE_ESCALATE=0: the two-pass schedule)
    inline = (be.hip and cfg.inline_escalate and cfg.escalate_budget > cfg.node_budget and cfg.escalate_max_open > 0
              and not esc_after_relu
              and os.environ.get("FAIRIFY_INLINE_ESCALATE", "1") != "0" and os.environ.get("FAIRIFY_TORCH_BAB") != "1")
    solver = BaBSolver(be, q, BaBConfig(node_budget=cfg.node_budget, batch_nodes=cfg.batch_nodes,
                                        time_budget=budget,
                                        escalate_budget=cfg.escalate_budget if inline else 0,
                                        escalate_max_w=cfg.escalate_max_open if inline else 0,
                                        escalate_steps=tuple(cfg.escalate_probation) if inline else ()), timer=tm)
    with tm("bab"):
        res = solver.solve(lo_np, hi_np, mlp, init_status=status)
    newly_sat = (res.status == SAT) & (status != SAT)
    stage[newly_sat] = "bab"
    stage[(res.status == UNSAT)] = "bab"
    cex_x[newly_sat] = res.cex_x[newly_sat]
    cex_xp[newly_sat] = res.cex_xp[newly_sat]
    status = res.status.copy()
    nodes = res.nodes.copy()
    # node expansions per stage (STAGE_NODE_COLS; bench JSON / diagnostics): each stage's delta of `nodes`
    stage_nodes = np.zeros((Pn, len(STAGE_NODE_COLS)), dtype=np.int64)
    stage_nodes[:, 0] = res.nodes

    def charge(col: int, before: np.ndarray) -> None:
        stage_nodes[:, col] += (nodes - before).astype(np.int64)

    open_left = res.open_left
    forced = faults.forced_unknown(ids) & (stage == "bab")      # fault injection: solver "timeouts"
    if forced.any():
        status[forced] = UNKNOWN
        stage[forced] = ""
        cex_x[forced] = 0
        cex_xp[forced] = 0
    sync()
    t_bab = time.time() - t0

    # ---------------- stage 3a: residual falsifier (heavy sampling + lattice local search) on
    # the partitions the BaB left UNKNOWN; candidates are confirmed exactly
    if cfg.residual_samples > 0:
        unk = np.nonzero(status == UNKNOWN)[0]
        if unk.size:
            t0 = time.time()
            with tm("falsify"):
                ut = torch.from_numpy(unk).to(dev)
                fr = residual_falsify(be, q, lo[ut], hi[ut], pids[ut], values, pairs, cfg.seed,
                                      n_samples=cfg.residual_samples, k_starts=cfg.residual_starts,
                                      iters=cfg.residual_iters)
                fnd = fr.found.cpu().numpy()
                if fnd.any():
                    fi = np.nonzero(fnd)[0]
                    X = fr.wit_x[fi].cpu().numpy().round().astype(np.int64)
                    XP = fr.wit_xp[fi].cpu().numpy().round().astype(np.int64)
                    pi = unk[fi]
                    ok = exact.check_pair_constraints(X, XP, lo_np[pi], hi_np[pi], q.pa_idx, q.ra_idx, q.tau)
                    viol = exact.is_violation(mlp, X, XP) & ok
                    hit = pi[viol]
                    status[hit] = SAT
                    cex_x[hit], cex_xp[hit] = X[viol], XP[viol]
                    stage[hit] = "falsify"
            sync()
            t_bab += time.time() - t0

    # ---------------- stage 3b: escalated sound BaB passes on what is still UNKNOWN (the cheap
    # first pass decides the bulk; only residue partitions whose open frontier stayed small -- the
    # ones a deeper search can still close -- pay for the deep budgets).  relu_first: after 3r.
    stages = []
    if cfg.escalate_budget > cfg.node_budget and not inline:
        stages.append((cfg.escalate_budget, cfg.escalate_max_open))
    stages += [tuple(st) for st in cfg.escalate_stages]
    prev_budget = cfg.escalate_budget if inline else cfg.node_budget

    def escalate():
        nonlocal prev_budget, open_left, t_bab
        for e_budget, e_open in stages:
            if e_budget <= prev_budget:
                continue
            prev_budget = e_budget
            want = (status == UNKNOWN) & ~forced
            if e_open > 0 and open_left is not None:
                want &= open_left <= e_open
            unk = np.nonzero(want)[0]
            if not unk.size:
                continue
            t0 = time.time()
            el = time.time() - t_start
            esolver = BaBSolver(be, q, BaBConfig(node_budget=e_budget, batch_nodes=cfg.batch_nodes,
                                                 time_budget=max(0.0, budget - el)), timer=tm)
            with tm("bab.escalate"):
                eres = esolver.solve(lo_np[unk], hi_np[unk], mlp)
            dec_e = np.isin(eres.status, (SAT, UNSAT))
            hit = unk[dec_e]
            status[hit] = eres.status[dec_e]
            stage[hit] = "bab"
            es = eres.status == SAT
            cex_x[unk[es]] = eres.cex_x[es]
            cex_xp[unk[es]] = eres.cex_xp[es]
            nodes[unk] += eres.nodes
            if open_left is not None and eres.open_left is not None:
                open_left = open_left.copy()
                open_left[unk] = eres.open_left
            sync()
            t_bab += time.time() - t0

    if not esc_after_relu:
        n0_ = nodes.copy()
        escalate()
        charge(0, n0_)

    # ---------------- stage 3r: ReLU-phase branch-and-bound on the residue (rigorous GPU bounds
    # with neuron-phase splits: the exact-zero partitions input splitting cannot close)
    if relu_on:
        from .relu_bab import ReluBaBSolver, ReluConfig

        unk = np.nonzero((status == UNKNOWN) & ~forced)[0]
        n0_ = nodes.copy()
        if unk.size:
            t0 = time.time()
            el = time.time() - t_start
            rsolver = ReluBaBSolver(be, q, ReluConfig(node_budget=cfg.relu_budget, batch_nodes=cfg.batch_nodes,
                                                      time_budget=max(0.0, budget - el)), timer=tm)
            with tm("relu"):
                rres = rsolver.solve(lo_np[unk], hi_np[unk], mlp)
            dec_r = np.isin(rres.status, (SAT, UNSAT))
            hit = unk[dec_r]
            status[hit] = rres.status[dec_r]
            stage[hit] = "relu"
            rs = rres.status == SAT
            cex_x[unk[rs]] = rres.cex_x[rs]
            cex_xp[unk[rs]] = rres.cex_xp[rs]
            nodes[unk] += rres.nodes
            sync()
            t_bab += time.time() - t0
        charge(1, n0_)
    # ---------------- stage 3b': beta-CROWN phase-split BaB on the residue (the wide nets' UNSAT
    # partitions need phase splits as constraints on the region: Lagrangian split multipliers)
    if beta_on:
        unk = np.nonzero((status == UNKNOWN) & ~forced)[0]
        if unk.size:
            t0 = time.time()
            el = time.time() - t_start
            n0_ = nodes.copy()
            with tm("beta"):
                _beta_round(be, q, mlp, unk, lo_np, hi_np, cfg.beta_budget, max(0.0, budget - el), cfg.batch_nodes,
                            status, stage, cex_x, cex_xp, nodes, tm, probe_levels=cfg.beta_probe_levels, cfg=cfg)
            charge(2, n0_)
            sync()
            t_bab += time.time() - t0
    if esc_after_relu:
        n0_ = nodes.copy()
        escalate()
        charge(0, n0_)

    # ---------------- stage 3c: exact host solver on the residue (the reference's Z3 check,
    # src/AC/Verify-AC.py:145-158): Z3 when installed, else the HiGHS MILP back-end fed the
    # GPU's rigorous layer bounds (smt/milp.py); no-op with "none"
    t_smt = 0.0
    if cfg.smt_backend != "none":
        from ..smt import solver as smt_solver

        backend = smt_solver.resolve(cfg.smt_backend)
        unk = np.nonzero((status == UNKNOWN) & ~forced)[0]
        if backend == "milp" and unk.size and cfg.anytime_seconds <= 0:   # anytime: rounds inside 3d
            t0 = time.time()
            if _use_lp(cfg, q):
                with tm("lp"):
                    _lp_round(be, mlp, q, unk, lo_np, hi_np, values_np, pairs_np, cfg.lp_budget,
                              cfg.smt_timeout or cfg.soft_timeout, cfg.smt_workers, status, stage, cex_x, cex_xp)
            else:
                with tm("milp"):
                    _milp_round(be, mlp, q, unk, lo_np, hi_np, values_np, pairs_np,
                                cfg.smt_timeout or cfg.soft_timeout, cfg.smt_workers, status, stage, cex_x, cex_xp,
                                trust=cfg.trust_milp)
            t_smt = time.time() - t0
        elif backend != "milp":
            hs = _host_smt(cfg)
            if hs.active and unk.size:
                t0 = time.time()
                with tm("smt"):
                    ut = torch.from_numpy(unk).to(dev)
                    st_mask = ((code[ut][:, :Nh] & H.PM_ST) != 0) if fused else st_dead[ut][:, :Nh]
                    futs = hs.submit(mlp, q, lo_np[unk], hi_np[unk], st_mask)
                    for k, f in zip(unk, futs):
                        verdict, pair = f.result()
                        if verdict == "unsat":
                            status[k], stage[k] = UNSAT, "smt"
                        elif verdict == "sat" and pair is not None:
                            X = np.array([pair[0]], dtype=np.int64)
                            XP = np.array([pair[1]], dtype=np.int64)
                            ok = exact.check_pair_constraints(X, XP, lo_np[k:k + 1], hi_np[k:k + 1], q.pa_idx,
                                                              q.ra_idx, q.tau)
                            if ok[0] and exact.is_violation(mlp, X, XP)[0]:
                                status[k], stage[k] = SAT, "smt"
                                cex_x[k], cex_xp[k] = X[0], XP[0]
                t_smt = time.time() - t0
    t_bab += t_smt

    # ---------------- stage 3d: anytime escalation on the residue (sound; before the heuristic)
    anytime_rounds = 0
    n_any = nodes.copy()
    if cfg.anytime_seconds > 0:
        t0 = time.time()
        deadline = t0 + cfg.anytime_seconds
        e_budget = max(prev_budget, cfg.node_budget)
        n_samp = max(cfg.residual_samples, 1)
        use_milp = False
        if cfg.smt_backend != "none":
            from ..smt import solver as smt_solver

            use_milp = smt_solver.resolve(cfg.smt_backend) == "milp"
        milp_limit = cfg.anytime_milp_seconds
        # x growth per round; the first round at budget / 4: trained AC-7's UNSAT partitions need
        # 100-5 000 LP nodes (profiles/r4/lp_tree_sizes_ac7_trained.jsonl), and every round restarts
        # its searches from the root
        lp_div = cfg.anytime_lp_div or (1 if len(pairs_np) > 2 else 4)
        lp_budget = max(1, cfg.lp_budget // lp_div)
        relu_any = _relu_supported(q)
        r_budget = max(cfg.relu_budget, 1) if relu_on else 64      # x growth before the first round
        bab_live, relu_live = True, True                          # stages still yielding
        beta_any = cfg.anytime_beta > 0 and _beta_supported(q)     # any width in the anytime rounds
        beta_live = beta_any
        b_budget = max(cfg.anytime_beta // cfg.anytime_growth, 1) if not beta_on else max(cfg.beta_budget,
                                                                                         cfg.anytime_beta)
        with tm("anytime"):
            while True:
                unk = np.nonzero((status == UNKNOWN) & ~forced)[0]
                if not unk.size or time.time() >= deadline:
                    break
                anytime_rounds += 1
                # (b) beta-CROWN phase-split BaB with a growing budget first: it closes the wide nets'
                # UNSAT residue on the GPU in a few dozen nodes per partition, before the host LP
                # is handed what is left
                if beta_any and beta_live:
                    b_budget *= cfg.anytime_growth
                    left = deadline - time.time()
                    if left > 0:
                        # at most half of what is left: where it does not converge (random-init
                        # residue) the other stages keep their time
                        with tm("beta"):
                            ndec = _beta_round(be, q, mlp, unk, lo_np, hi_np, b_budget, 0.5 * left, cfg.batch_nodes,
                                               status, stage, cex_x, cex_xp, nodes, tm, cfg=cfg, anytime=True)
                        if ndec < cfg.anytime_min_yield * unk.size:
                            beta_live = False
                    unk = np.nonzero((status == UNKNOWN) & ~forced)[0]
                    if not unk.size:
                        break
                # (e, started first) verified-LP branch-and-bound on the host workers with a growing
                # node budget, CONCURRENT with this round's GPU stages (collected at the round's end):
                # on a residue the GPU stages do not converge on (trained AC-7) the round costs
                # max(GPU, LP) instead of their sum
                lp_pending = None
                if use_milp and _use_lp(cfg, q):
                    left = deadline - time.time()
                    with tm("lp.submit"):
                        lp_pending = _lp_submit(be, mlp, q, unk, lo_np, hi_np, values_np, pairs_np, lp_budget,
                                                min(milp_limit * 4, left), cfg.smt_workers, deadline=deadline)
                # (a) fresh samples + boundary walk + local search, new seed every round
                n_samp = min(n_samp * cfg.anytime_growth, cfg.anytime_max_samples)
                ut = torch.from_numpy(unk).to(dev)
                fr = residual_falsify(be, q, lo[ut], hi[ut], pids[ut], values, pairs,
                                      cfg.seed + 7919 * anytime_rounds, n_samples=n_samp,
                                      k_starts=2 * cfg.residual_starts, iters=2 * cfg.residual_iters)
                fnd = fr.found.cpu().numpy()
                if fnd.any():
                    fi = np.nonzero(fnd)[0]
                    X = fr.wit_x[fi].cpu().numpy().round().astype(np.int64)
                    XP = fr.wit_xp[fi].cpu().numpy().round().astype(np.int64)
                    pi = unk[fi]
                    ok = exact.check_pair_constraints(X, XP, lo_np[pi], hi_np[pi], q.pa_idx, q.ra_idx, q.tau)
                    viol = exact.is_violation(mlp, X, XP) & ok
                    hit = pi[viol]
                    status[hit] = SAT
                    cex_x[hit], cex_xp[hit] = X[viol], XP[viol]
                    stage[hit] = "falsify"
                # (c) deeper sound BaB, in groups that fit the node pool
                e_budget *= cfg.anytime_growth
                if e_budget > cfg.anytime_max_budget:
                    bab_live = False
                if not (bab_live or (relu_any and cfg.relu_budget > 0 and relu_live) or use_milp or beta_live):
                    break                                       # nothing left that can still decide
                unk = np.nonzero((status == UNKNOWN) & ~forced)[0]
                if _VERBOSE_ANYTIME:
                    print(f"[anytime] {mlp.name} round {anytime_rounds}: {unk.size} unknown after falsify "
                          f"({n_samp} samples), BaB budget {e_budget}, {deadline - time.time():.1f}s left",
                          flush=True)
                G = max(1, cfg.anytime_pool // e_budget)
                n_try = n_dec = 0
                for g0 in range(0, unk.size if bab_live else 0, G):
                    left = deadline - time.time()
                    if left <= 0:
                        break
                    grp = unk[g0:g0 + G]
                    asolver = BaBSolver(be, q, BaBConfig(node_budget=e_budget, batch_nodes=cfg.batch_nodes,
                                                         time_budget=left, max_pool=cfg.anytime_pool), timer=tm)
                    ares = asolver.solve(lo_np[grp], hi_np[grp], mlp)
                    dec_a = np.isin(ares.status, (SAT, UNSAT))
                    n_try += grp.size
                    n_dec += int(dec_a.sum())
                    hit = grp[dec_a]
                    status[hit] = ares.status[dec_a]
                    stage[hit] = "bab"
                    sa = ares.status == SAT
                    cex_x[grp[sa]] = ares.cex_x[sa]
                    cex_xp[grp[sa]] = ares.cex_xp[sa]
                    nodes[grp] += ares.nodes
                    if n_try >= 256 and n_dec < cfg.anytime_min_yield * n_try:
                        break                                   # not converging: stop the round early
                if bab_live and n_try and n_dec < cfg.anytime_min_yield * n_try:
                    bab_live = False
                # (d) ReLU-phase BaB with a growing budget, any layer width (the anytime budget pays
                # for the wide nets too; it re-proves partitions the MILP only claims)
                if relu_any and cfg.relu_budget > 0 and relu_live:
                    r_budget *= cfg.anytime_growth
                    unk = np.nonzero((status == UNKNOWN) & ~forced)[0]
                    left = deadline - time.time()
                    r_try = r_dec = 0
                    if unk.size and left > 0:
                        from .relu_bab import ReluBaBSolver, ReluConfig

                        G = max(1, cfg.anytime_pool // max(1, r_budget))
                        for g0 in range(0, unk.size, G):
                            left = deadline - time.time()
                            if left <= 0:
                                break
                            grp = unk[g0:g0 + G]
                            rs = ReluBaBSolver(be, q, ReluConfig(node_budget=r_budget, batch_nodes=cfg.batch_nodes,
                                                                 time_budget=left), timer=tm)
                            with tm("relu"):
                                rr = rs.solve(lo_np[grp], hi_np[grp], mlp)
                            dec_r = np.isin(rr.status, (SAT, UNSAT))
                            r_try += grp.size
                            r_dec += int(dec_r.sum())
                            status[grp[dec_r]] = rr.status[dec_r]
                            stage[grp[dec_r]] = "relu"
                            sr = rr.status == SAT
                            cex_x[grp[sr]] = rr.cex_x[sr]
                            cex_xp[grp[sr]] = rr.cex_xp[sr]
                            nodes[grp] += rr.nodes
                            if r_try >= 256 and r_dec < cfg.anytime_min_yield * r_try:
                                break
                    if r_try and r_dec < cfg.anytime_min_yield * r_try:
                        relu_live = False
                # (e) collect the verified-LP searches started with the round (sound UNSAT and SAT),
                # or -- trust_milp / lp_budget 0 -- the HiGHS MILP with a growing time limit
                if lp_pending is not None:
                    with tm("lp"):
                        _lp_collect(mlp, lp_pending, lp_budget, status, stage, cex_x, cex_xp)
                    lp_budget *= cfg.anytime_growth
                    milp_limit *= cfg.anytime_growth
                elif use_milp:
                    # partitions the MILP already claimed UNSAT (unverified) are not re-solved
                    unk = np.nonzero((status == UNKNOWN) & ~forced & (stage != "milp"))[0]
                    left = deadline - time.time()
                    if unk.size and left > 0:
                        with tm("milp"):
                            _milp_round(be, mlp, q, unk, lo_np, hi_np, values_np, pairs_np, min(milp_limit, left),
                                        cfg.smt_workers, status, stage, cex_x, cex_xp, deadline=deadline,
                                        trust=cfg.trust_milp)
                    milp_limit *= cfg.anytime_growth
        sync()
        t_bab += time.time() - t0

    # ---------------- stage 4: heuristic retry for UNKNOWN partitions (unsound, flagged)
    h_attempt = np.zeros(Pn, dtype=np.int64)
    h_success = np.zeros(Pn, dtype=np.int64)
    h_cnt = np.zeros(Pn, dtype=np.int64)
    t_cnt = st_cnt.copy()
    masked: Dict[int, np.ndarray] = {}
    t_heur = 0.0
    unk = np.nonzero(status == UNKNOWN)[0]
    charge(3, n_any)          # every anytime round (between n_any and here)
    n_h = nodes.copy()
    if cfg.heuristic and unk.size and ibp_ub is not None:
        t0 = time.time()
        h_attempt[unk] = 1
        with tm("heuristic.masks"):
            ut = torch.from_numpy(unk).to(dev)
            if fused:
                _, hm_t, hc_t = H.heuristic(be, ut, ibp_lb, ibp_ub, code, cfg.heuristic_p)
                md_np = hm_t.cpu().numpy().astype(bool)
                hc_np = hc_t.cpu().numpy().astype(np.int64)
                h_cnt[unk], t_cnt[unk] = hc_np[:, 0], hc_np[:, 1]
                dead_t = hm_t[:, :Nh].contiguous()
            else:
                hd_t, md_t = P_.heuristic_prune_batch(ibp_lb[ut], ibp_ub[ut], cand[ut], s_cand[ut], st_dead[ut],
                                                      widths, cfg.heuristic_p)
                md_np = md_t.cpu().numpy()
                h_cnt[unk] = hd_t.sum(dim=1).cpu().numpy()
                t_cnt[unk] = md_np.sum(axis=1)
                dead_t = torch.from_numpy(md_np[:, :Nh]).to(dev)
            for k, p in enumerate(unk):
                masked[p] = md_np[k]
        # partitions whose heuristic mask equals the sound mask would re-run the same query
        sub_lo, sub_hi = lo_np[unk], hi_np[unk]
        exact_models = _LazyMasked(mlp, [masked[p] for p in unk], widths)
        hsolver = BaBSolver(be, q, BaBConfig(node_budget=cfg.heuristic_node_budget, batch_nodes=cfg.batch_nodes,
                                             time_budget=budget), dead=dead_t, timer=tm)
        with tm("heuristic.bab"):
            hres = hsolver.solve(sub_lo, sub_hi, mlp, exact_models=exact_models)
        dec = np.isin(hres.status, (SAT, UNSAT))
        hp = unk[dec]
        h_success[hp] = 1
        status[hp] = hres.status[dec]
        stage[hp] = "heuristic"
        hs = unk[hres.status == SAT]
        cex_x[hs] = hres.cex_x[hres.status == SAT]
        cex_xp[hs] = hres.cex_xp[hres.status == SAT]
        if hs.size:
            # a heuristic SAT pair was confirmed on the MASKED net; one that also flips the original
            # network (the reference's V-accurate replay, src/AC/Verify-AC.py:225-258) is a sound
            # counterexample: stage "heuristic-confirmed"
            ok = exact.check_pair_constraints(cex_x[hs], cex_xp[hs], lo_np[hs], hi_np[hs], q.pa_idx, q.ra_idx, q.tau)
            real = exact.is_violation(mlp, cex_x[hs], cex_xp[hs]) & ok
            stage[hs[real]] = "heuristic-confirmed"
        nodes[unk] += hres.nodes
        charge(4, n_h)
        sync()
        t_heur = time.time() - t0

    # ---------------- K6: final dead-neuron masks as packed bitsets (optional)
    mask_bits = None
    if cfg.keep_masks:
        with tm("masks"):
            mask_bits = _final_mask_bits(be, mlp, code if fused else None, None if fused else st_dead, masked, unk,
                                         hm_t if (fused and masked) else None, Pn)

    # ---------------- stage 5: replay / fidelity (batched on the device)
    t0 = time.time()
    with tm("replay"):
        sat_idx = np.nonzero(status == SAT)[0]
        c_check = np.zeros(Pn, dtype=np.int64)
        v_acc = np.zeros(Pn, dtype=np.int64)
        if sat_idx.size:
            xo = mlp.predict(cex_x[sat_idx])
            xpo = mlp.predict(cex_xp[sat_idx])
            v_acc[sat_idx] = (xo != xpo).astype(np.int64)
            dmask = np.zeros((sat_idx.size, Nh), dtype=bool)
            for k, p in enumerate(sat_idx):
                if p in masked:
                    dmask[k] = masked[p][:Nh]
            xt = torch.from_numpy(np.concatenate([cex_x[sat_idx], cex_xp[sat_idx]])).to(dev, torch.float32)
            dt_ = torch.from_numpy(np.concatenate([dmask, dmask])).to(dev)
            zp = be.forward(xt, dt_).cpu().numpy()
            c1 = (zp[:sat_idx.size] > 0).astype(np.int64)
            c2 = (zp[sat_idx.size:] > 0).astype(np.int64)
            c_check[sat_idx] = ((c1 == xo) & (c2 == xpo)).astype(np.int64)
        agree = np.full(Pn, cfg.sim_size, dtype=np.int64)     # Pruned-acc numerator
        tp = np.zeros(Pn, dtype=np.int64)                      # Pruned-F1 counts (pruned_metrics)
        fp = np.zeros(Pn, dtype=np.int64)
        if masked or cfg.pruned_metrics:
            # pruned_metrics: every partition (unmasked ones with their sound-pruned net, which
            # equals the original on the box: mask of zeros) for the experiment drivers' F1
            hp = np.arange(Pn) if cfg.pruned_metrics else np.array(sorted(masked))
            dm_np = np.zeros((hp.size, Nh), dtype=np.uint8)
            for k, p in enumerate(hp):
                if p in masked:
                    dm_np[k] = masked[p][:Nh]
            dm = torch.from_numpy(dm_np).to(dev)
            ag = None
            if be.hip and os.environ.get("FAIRIFY_FUSED_PRUNE", "1") != "0":
                from ..ops import hip as H

                ag = H.agree(be, torch.from_numpy(hp).to(dev), lo, hi, pids, dm, cfg.sim_size, cfg.seed)
            if ag is not None:
                ag_np = ag.cpu().numpy().astype(np.int64)
                agree[hp], tp[hp], fp[hp] = ag_np[:, 0], ag_np[:, 1], ag_np[:, 2]
            else:
                from ..ops.reference import sample_points

                X = sample_points(lo[hp], hi[hp], pids[hp], cfg.sim_size, cfg.seed)
                z0 = be.forward(X)
                z1 = be.forward(X, dm.bool()[:, None, :].expand(-1, X.shape[1], -1))
                agree[hp] = ((z0 > 0) == (z1 > 0)).sum(dim=1).cpu().numpy()
                tp[hp] = ((z0 > 0) & (z1 > 0)).sum(dim=1).cpu().numpy()
                fp[hp] = ((z0 <= 0) & (z1 > 0)).sum(dim=1).cpu().numpy()
    t_replay = time.time() - t0

    # ---------------- records: dead-neuron counts, work, per-chunk stage times (the per-partition
    # time columns are apportioned from these by derive_columns, here and after a gather)
    verdict = np.where(status == SAT, "sat", np.where(status == UNSAT, "unsat", "unknown"))
    stage_f = np.where(stage == "", np.where(verdict != "unknown", "bab", ""), stage)
    core = dict(
        grid_id=np.asarray(ids, dtype=np.int64), verdict=verdict, stage=stage_f.astype(object),
        h_attempt=h_attempt, h_success=h_success,
        b_cnt=b_cnt, s_cnt=s_cnt, st_cnt=st_cnt, h_cnt=h_cnt, t_cnt=t_cnt, agree=agree, tp=tp, fp=fp, nodes=nodes.astype(np.int64),
        c_check=c_check, v_accurate=v_acc, cex_x=cex_x, cex_xp=cex_xp)
    core["stage_nodes"] = stage_nodes
    if mask_bits is not None:
        core["mask_bits"] = mask_bits
    return core, (Pn, t_sim + t_prune + t_bab, t_bab, t_heur, t_replay)


def _final_mask_bits(be, mlp: MLP, code, st_dead, masked: Dict[int, np.ndarray], unk: np.ndarray, hm_t, Pn: int
                     ) -> np.ndarray:
    """[Pn, ceil(N/8)] uint8 (numpy.packbits order) final dead masks: the sound-prune mask
    (ST = B ∪ S with one neuron kept alive per layer), replaced by the merged heuristic mask for
    the partitions of the heuristic retry -- the mask whose popcount is the CSV's T-compression
    numerator.  On the GPU the mask algebra codes are packed by ``fa_pack_masks_kernel``."""
    N = mlp.n_neurons
    if code is not None and be.hip:
        from ..ops import hip as H

        fm = ((code & H.PM_ST) != 0).to(torch.uint8)
        if hm_t is not None and len(unk):
            fm[torch.from_numpy(np.asarray(unk)).to(fm.device)] = (hm_t != 0).to(torch.uint8)
        bits, _ = H.pack_masks(fm)
        return bits.cpu().numpy()
    m = np.zeros((Pn, N), dtype=bool) if st_dead is None else st_dead.cpu().numpy().astype(bool)
    for p, mk in masked.items():
        m[p] = np.asarray(mk, dtype=bool)[:N]
    return np.packbits(m, axis=1)


class StreamPool:
    """Host threads, each driving its own HIP stream, that verify several chunks of one model
    concurrently (the native BaB level loop releases the GIL, so one chunk's host phases and
    synchronisations overlap the other chunks' kernels).  ``workers == 1`` runs inline."""

    def __init__(self, device: torch.device, workers: int):
        import threading
        from concurrent.futures import ThreadPoolExecutor

        self.device = torch.device(device)
        self.workers = max(1, int(workers))
        self._tls = threading.local()
        self._pool = ThreadPoolExecutor(max_workers=self.workers) if self.workers > 1 else None

    def _stream_ctx(self):
        import contextlib

        if self.device.type != "cuda":
            return contextlib.nullcontext()
        if getattr(self._tls, "stream", None) is None:
            self._tls.stream = torch.cuda.Stream(self.device)
        return torch.cuda.stream(self._tls.stream)

    def run(self, fn: Callable, items: Sequence) -> List:
        """``[fn(item) for item in items]``, concurrently, results in item order."""
        def one(it):
            with self._stream_ctx():
                out = fn(it)
                if self.device.type == "cuda":
                    torch.cuda.current_stream(self.device).synchronize()
            return out

        if self._pool is None or len(items) <= 1:
            return [one(it) for it in items]
        return [f.result() for f in [self._pool.submit(one, it) for it in items]]

    def close(self):
        if self._pool is not None:
            self._pool.shutdown(wait=True)


def concat_records(parts: Sequence["ChunkRecords"]) -> "ChunkRecords":
    parts = [p for p in parts if len(p)]
    if not parts:
        raise ValueError("no records")
    if len(parts) == 1:
        return parts[0]
    keys = [k for k in parts[0].core if all(k in p.core for p in parts)]
    core = {k: np.concatenate([p.core[k] for p in parts]) for k in keys}
    segs = [sg for p in parts for sg in p.segments]
    return ChunkRecords(core, parts[0].orig_acc, segments=segs, n_neurons=parts[0].n_neurons,
                        sim_size=parts[0].sim_size)


# node expansions per stage (core["stage_nodes"] columns): input-split BaB with its escalation, the
# ReLU-phase BaB, the fixed beta pass, every anytime round, the heuristic retry
STAGE_NODE_COLS = ("bab", "relu", "beta", "anytime", "heuristic")
CORE_COLUMNS = ("grid_id", "verdict", "stage", "h_attempt", "h_success", "b_cnt", "s_cnt", "st_cnt", "h_cnt",
                "t_cnt", "agree", "tp", "fp", "nodes", "c_check", "v_accurate", "cex_x", "cex_xp")


def derive_columns(core: Dict[str, np.ndarray], segments, n_neurons: int, sim_size: int) -> Dict[str, np.ndarray]:
    """The 24-column CSV quantities from the per-partition core columns.

    Compressions = dead counts / N (output neuron included, utils/prune.py:194-203); Pruned-acc
    = agreeing simulation points / sim_size; the stage times of every chunk segment
    ``(n, t_sim+prune+bab, t_bab, t_heur, t_replay)`` are apportioned over its partitions by
    work (BaB node expansions).  Pure function of its inputs, so rank 0 reproduces exactly what
    the producing rank would have written."""
    N = float(max(1, n_neurons))
    h = core["h_attempt"] > 0
    out = dict(core)
    out["b_comp"] = core["b_cnt"] / N
    out["s_comp"] = core["s_cnt"] / N
    out["st_comp"] = core["st_cnt"] / N
    out["h_comp"] = np.where(h, core["h_cnt"] / N, 0.0)
    out["t_comp"] = core["t_cnt"] / N
    out["pruned_acc"] = core["agree"] / float(max(1, sim_size))
    # F1 of the pruned net's labels against the original's on the simulation points (sklearn
    # f1_score(sim_y_orig, sim_y), zero_division -> 0): fn = S - agree - fp
    if "tp" in core:
        tp_, fp_ = core["tp"].astype(np.float64), core["fp"].astype(np.float64)
        fn_ = float(sim_size) - core["agree"] - fp_
        den = 2 * tp_ + fp_ + fn_
        out["pruned_f1"] = np.where(den > 0, 2 * tp_ / np.maximum(den, 1), 0.0)
    n = len(core["verdict"])
    s_t, sv_t, hv_t, rp_t = (np.zeros(n) for _ in range(4))
    off = 0
    for cnt, t_spb, t_bab, t_heur, t_rep in segments:
        cnt = int(cnt)
        sl = slice(off, off + cnt)
        work = core["nodes"][sl]
        s_t[sl] = _amortize(t_spb, work)
        sv_t[sl] = _amortize(t_bab, work)
        if t_heur > 0:
            hv_t[sl] = _amortize(t_heur, np.where(h[sl], work, 0))
        rp_t[sl] = _amortize(t_rep, np.zeros(cnt))
        off += cnt
    if off != n:
        raise ValueError(f"segments cover {off} partitions, records hold {n}")
    out["sv_time"], out["s_time"], out["hv_time"], out["h_time"] = sv_t, s_t, hv_t, hv_t
    out["total_time"] = s_t + hv_t + rp_t
    return out


class ChunkRecords(Sequence):
    """Per-partition results of one or more chunks, stored column-wise (numpy arrays).

    ``core`` holds what a rank ships (verdicts, stages, dead counts, work, counterexamples),
    ``segments`` the per-chunk stage times; ``cols`` adds the derived CSV quantities.  Behaves
    like a list of per-partition dicts (the CSV/runner view, built lazily per row)."""

    _INT = ("grid_id", "h_attempt", "h_success", "c_check", "v_accurate", "nodes")
    _HIDE = ("cex_x", "cex_xp", "b_cnt", "s_cnt", "st_cnt", "h_cnt", "t_cnt", "agree", "tp", "fp", "pruned_f1",
             "mask_bits", "stage_nodes")

    def __init__(self, core: Dict[str, np.ndarray], orig_acc: Optional[float] = None, segments=None,
                 n_neurons: int = 1, sim_size: int = 1):
        self.core = core
        self.orig_acc = orig_acc
        self.segments = list(segments) if segments is not None else [(len(core["verdict"]), 0.0, 0.0, 0.0, 0.0)]
        self.n_neurons = n_neurons
        self.sim_size = sim_size
        self.cols = derive_columns(core, self.segments, n_neurons, sim_size)

    def __len__(self) -> int:
        return len(self.cols["verdict"])

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(len(self)))]
        c = self.cols
        sat = c["verdict"][i] == "sat"
        d = {k: (int(v[i]) if k in self._INT else (str(v[i]) if v.dtype.kind in "OU" else float(v[i])))
             for k, v in c.items() if k not in self._HIDE}
        d["orig_acc"] = self.orig_acc
        d["c1"] = c["cex_x"][i].astype(np.float32) if sat else None
        d["c2"] = c["cex_xp"][i].astype(np.float32) if sat else None
        return d

    def counts(self) -> Dict[str, int]:
        v = self.cols["verdict"]
        return {"sat": int((v == "sat").sum()), "unsat": int((v == "unsat").sum()),
                "unknown": int((v == "unknown").sum())}


def sample_host(lo: np.ndarray, hi: np.ndarray, pid: int, n_samples: int, seed: int) -> np.ndarray:
    from ..ops.reference import sample_points

    X = sample_points(torch.from_numpy(lo[None]).float(), torch.from_numpy(hi[None]).float(),
                      torch.tensor([pid]), n_samples, seed)
    return X[0].numpy().astype(np.int64)


def verify_model(mlp: MLP, q: ResolvedQuery, grid: Grid, order: np.ndarray, cfg: VerifyConfig,
                 device="cpu", orig_acc: Optional[float] = None,
                 on_chunk: Optional[Callable[[List[PartitionRecord]], None]] = None,
                 max_partitions: Optional[int] = None) -> ModelRun:
    """Verify partitions of ``grid`` in ``order`` (ids) until done or the hard timeout."""
    be = Backend(mlp, device=device)
    run = ModelRun(model=mlp.name)
    t0 = time.time()
    total = len(order) if max_partitions is None else min(len(order), max_partitions)
    pos = 0
    while pos < total:
        elapsed = time.time() - t0
        if elapsed > cfg.hard_timeout:
            run.stopped_by_hard_timeout = True
            break
        ids = order[pos:min(total, pos + cfg.chunk)]
        recs = verify_chunk(be, mlp, q, grid, ids, cfg, orig_acc=orig_acc,
                            time_budget=cfg.hard_timeout - elapsed)
        out = []
        for r in recs:
            out.append(PartitionRecord(partition_id=pos + len(out) + 1, **r))
        run.records.extend(out)
        pos += len(ids)
        if on_chunk is not None:
            on_chunk(out)
    run.attempted = len(run.records)
    run.wall = time.time() - t0
    return run
