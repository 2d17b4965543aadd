"""Thin Python wrappers launching the HIP kernels of ``fairify_amd._C`` on torch's stream.

Every wrapper allocates its outputs with torch (caching allocator, current device), checks
shapes/dtypes/contiguity on the host before launch (a mis-shaped launch must never reach the
GPU), and passes raw pointers + ``torch.cuda.current_stream().cuda_stream``.
"""
from __future__ import annotations

import os
import threading
from typing import Optional, Sequence

import torch

from . import ext
from . import reference as ref


def _stream(dev) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


# Per-backend / per-grid lazy device state is created under this lock: the runner's worker threads share
# one Backend per model, and a second thread that built its own copy and published it over the first
# freed the first thread's tensor while a native runtime still held its device pointer (the beta
# runtime's transposed weights: whole chunks of beta roots bounded with freed memory, exp R6 W/X).
_LAZY_LOCK = threading.Lock()


def _net(be):
    n = getattr(be, "_hipnet", None)
    if n is None:
        with _LAZY_LOCK:
            n = getattr(be, "_hipnet", None)
            if n is None:
                dims = [be.mlp.n_in] + be.mlp.widths
                n = ext().Net(dims, be.unit)
                assert n.total_floats == be.flat.numel(), (n.total_floats, be.flat.numel())
                be._hipnet = n
    return n


def _c(t: torch.Tensor, dtype, shape=None, name="tensor") -> torch.Tensor:
    if t.dtype != dtype:
        t = t.to(dtype)
    t = t.contiguous()
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")
    return t


def _fold_mask(fold: Sequence[int], n0: int) -> int:
    m = 0
    for d in fold:
        if not 0 <= int(d) < min(n0, 64):
            raise ValueError(f"fold dim {d} out of range")
        m |= 1 << int(d)
    return m


def _ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


# ------------------------------------------------------------------------------------------------
def decode(grid, ids: torch.Tensor):
    """K1: grid-linear partition ids (int64, on the device) -> boxes ``lo, hi`` float32 [P, n0]
    decoded by ``fa_decode_kernel`` (the chunk tables are uploaded once per grid and device)."""
    dev = ids.device
    ids = _c(ids, torch.int64, (ids.shape[0],), "ids")
    tabs = grid.__dict__.setdefault("_dev_decode", {})
    key = str(dev)
    if key not in tabs:
        with _LAZY_LOCK:
            if key not in tabs:
                d = grid.decode_desc()
                cl = torch.from_numpy(d["chunk_lo"]).to(dev) if d["chunk_lo"].size else torch.zeros(1, device=dev)
                ch = torch.from_numpy(d["chunk_hi"]).to(dev) if d["chunk_hi"].size else torch.zeros(1, device=dev)
                torch.cuda.current_stream(dev).synchronize()     # published tables are complete for every stream
                tabs[key] = (d, cl, ch)
    d, cl, ch = tabs[key]
    n0 = int(d["radix"].shape[0])
    Pn = int(ids.shape[0])
    lo = torch.empty(Pn, n0, dtype=torch.float32, device=dev)
    hi = torch.empty(Pn, n0, dtype=torch.float32, device=dev)
    if Pn:
        ext().decode(d["radix"].tolist(), d["div"].tolist(), d["chunk_off"].tolist(), d["base_lo"].tolist(),
                     d["base_hi"].tolist(), ids.data_ptr(), Pn, cl.data_ptr(), ch.data_ptr(), lo.data_ptr(),
                     hi.data_ptr(), _stream(dev))
    return lo, hi


def pack_masks(masks: torch.Tensor, sel: int = 0xFF):
    """K6: [P, N] uint8 masks (dead where ``mask & sel``) -> (packed [P, ceil(N/8)] uint8 in
    ``numpy.packbits`` order, row hashes [P] int64) via ``fa_pack_masks_kernel``."""
    m = _c(masks, torch.uint8, name="masks")
    if m.dim() != 2:
        raise ValueError("masks: expected [P, N]")
    Pn, N = m.shape
    NB = (N + 7) // 8
    out = torch.empty(Pn, NB, dtype=torch.uint8, device=m.device)
    hsh = torch.empty(Pn, dtype=torch.int64, device=m.device)
    if Pn and N:
        ext().pack_masks(m.data_ptr(), Pn, N, N, int(sel), out.data_ptr(), NB, hsh.data_ptr(), _stream(m.device))
    return out, hsh


KNN_K = (1, 2, 3, 4, 5, 6, 7, 8, 10, 16)


def knn(X: torch.Tensor, k: int):
    """K10: indices [n, k] int32 of every row's k nearest rows of ``X`` (squared Euclidean, the
    row itself first, ties to the lower index) and their squared distances (``fa_knn_kernel``)."""
    X = _c(X, torch.float32, name="X")
    n, d = X.shape
    if not 1 <= d <= 64 or k not in KNN_K or k > n:
        raise ValueError(f"knn: unsupported shape n={n} d={d} k={k}")
    idx = torch.empty(n, k, dtype=torch.int32, device=X.device)
    dist = torch.empty(n, k, dtype=torch.float32, device=X.device)
    ext().knn(X.data_ptr(), n, d, k, idx.data_ptr(), dist.data_ptr(), _stream(X.device))
    return idx, dist


def activation_delta_sum(be, x: torch.Tensor, xp: torch.Tensor) -> torch.Tensor:
    """K13: sum over pairs of |act(x) - act(x')| per neuron [N] (hidden ReLU outputs, then the
    logit) via ``fa_actdiff_kernel``."""
    P_ = x.shape[0]
    x = _c(x, torch.float32, (P_, be.n0), "x")
    xp = _c(xp, torch.float32, (P_, be.n0), "xp")
    out = torch.zeros(be.mlp.n_neurons, dtype=torch.float32, device=x.device)
    if P_:
        ext().actdiff(_net(be), be.flat.data_ptr(), x.data_ptr(), xp.data_ptr(), P_, out.data_ptr(),
                      _stream(x.device))
    return out


def trace_marker(dev, tag: int) -> None:
    """Launch ``fa_trace_marker_kernel`` (a named one-thread kernel) on the current stream: the
    kernel trace's time-window delimiter (tools/trace_busy.py --window)."""
    ext().trace_marker(int(tag), 0, _stream(dev))


# ------------------------------------------------------------------------------------------------
def forward(be, x: torch.Tensor, dead: Optional[torch.Tensor] = None) -> torch.Tensor:
    shp = x.shape[:-1]
    x2 = _c(x.reshape(-1, be.n0), torch.float32, name="x")
    B = x2.shape[0]
    out = torch.empty(B, dtype=torch.float32, device=x.device)
    if B == 0:
        return out.view(shp)
    d = None
    if dead is not None:
        d = _c(dead.reshape(-1, be.n_hidden), torch.uint8, (B, be.n_hidden), "dead")
    ext().forward(_net(be), be.flat.data_ptr(), x2.data_ptr(), B, _ptr(d), out.data_ptr(), _stream(x.device))
    return out.view(shp)


def activation_counts(be, x: torch.Tensor) -> torch.Tensor:
    # generic rows: run the forward per layer through the reference on-device (rarely used on the
    # GPU path; the fused sim kernel counts activations itself)
    return ref.activation_counts(be.ws, be.bs, x)


# ------------------------------------------------------------------------------------------------
def point_bounds(be, x: torch.Tensor, dead: Optional[torch.Tensor] = None):
    R = x.shape[0]
    x2 = _c(x, torch.float32, (R, be.n0), "x")
    lb = torch.empty(R, dtype=torch.float32, device=x.device)
    ub = torch.empty(R, dtype=torch.float32, device=x.device)
    d = None
    if dead is not None:
        d = _c(dead, torch.uint8, (R, be.n_hidden), "dead")
    if R:
        ext().point_bounds(_net(be), be.flat.data_ptr(), x2.data_ptr(), _ptr(d), R, lb.data_ptr(), ub.data_ptr(),
                           _stream(x.device))
    return lb, ub


# ------------------------------------------------------------------------------------------------
def bounds(be, lo: torch.Tensor, hi: torch.Tensor, mode: str = "symbolic", dead: Optional[torch.Tensor] = None,
           keep_layers: bool = False, G: int = 0, fold: Sequence[int] = (),
           phase: Optional[torch.Tensor] = None) -> ref.BoundResult:
    """``fold``: input dims with lo == hi in EVERY row (folded into the constant column of the
    register-resident symbolic kernel; the caller guarantees degeneracy)."""
    R, n0 = lo.shape
    if n0 != be.n0:
        raise ValueError(f"box width {n0} != network input {be.n0}")
    dev = lo.device
    lo = _c(lo, torch.float32, (R, n0), "lo")
    hi = _c(hi, torch.float32, (R, n0), "hi")
    sym = 1 if mode == "symbolic" else 0
    f32 = dict(dtype=torch.float32, device=dev)
    out_lb = torch.empty(R, **f32)
    out_ub = torch.empty(R, **f32)
    res = ref.BoundResult(out_lb=out_lb, out_ub=out_ub)
    forms = [None] * 6
    if sym:
        res.Lc = torch.empty(R, n0, **f32)
        res.L0 = torch.empty(R, **f32)
        res.Le = torch.empty(R, **f32)
        res.Uc = torch.empty(R, n0, **f32)
        res.U0 = torch.empty(R, **f32)
        res.Ue = torch.empty(R, **f32)
        forms = [res.Lc, res.L0, res.Le, res.Uc, res.U0, res.Ue]
    N = be.mlp.n_neurons
    lay_lb = lay_ub = None
    if keep_layers:
        lay_lb = torch.empty(R, N, **f32)
        lay_ub = torch.empty(R, N, **f32)
    dead_out = torch.empty(R, be.n_hidden, dtype=torch.uint8, device=dev) if be.n_hidden else None
    d = None
    if dead is not None:
        d = _c(dead, torch.uint8, (R, be.n_hidden), "dead")
    ph = infeas = None
    if phase is not None:
        ph = _c(phase, torch.int8, (R, be.n_hidden), "phase")
        infeas = torch.zeros(R, dtype=torch.uint8, device=dev)
    if R:
        ext().bounds(_net(be), be.flat.data_ptr(), lo.data_ptr(), hi.data_ptr(), _ptr(d), R, sym,
                     out_lb.data_ptr(), out_ub.data_ptr(), *[_ptr(t) for t in forms],
                     _ptr(lay_lb), _ptr(lay_ub), _ptr(dead_out), G, _stream(dev), _fold_mask(fold, n0),
                     _ptr(ph), _ptr(infeas))
    if infeas is not None:
        res.infeasible = infeas.bool()
    if keep_layers:
        widths = be.mlp.widths
        offs = [0]
        for w in widths:
            offs.append(offs[-1] + w)
        res.layer_lb = [lay_lb[:, offs[i]:offs[i + 1]] for i in range(len(widths))]
        res.layer_ub = [lay_ub[:, offs[i]:offs[i + 1]] for i in range(len(widths))]
        res.lay_lb_full, res.lay_ub_full = lay_lb, lay_ub
    if dead_out is not None:
        res.dead_u8 = dead_out
        res.dead = dead_out.view(torch.bool)
    return res


# ------------------------------------------------------------------------------------------------
def crown(be, lo: torch.Tensor, hi: torch.Tensor, res: ref.BoundResult, dead: Optional[torch.Tensor] = None):
    """Backward output bounds (csrc/crown.hip) refining ``res`` in place: ``res`` must come from
    :func:`bounds` with mode='symbolic' and keep_layers=True on the same rows."""
    R, n0 = lo.shape
    N = be.mlp.n_neurons
    if res.Lc is None or res.layer_lb is None:
        raise ValueError("crown needs symbolic bounds with keep_layers=True")
    lo = _c(lo, torch.float32, (R, n0), "lo")
    hi = _c(hi, torch.float32, (R, n0), "hi")
    lay_lb = torch.cat(res.layer_lb, dim=1).contiguous() if isinstance(res.layer_lb, list) else res.layer_lb
    lay_ub = torch.cat(res.layer_ub, dim=1).contiguous() if isinstance(res.layer_ub, list) else res.layer_ub
    if lay_lb.shape[1] != N:          # keep_layers splits off the output neuron: append a pad column
        pad = torch.zeros(R, N - lay_lb.shape[1], dtype=torch.float32, device=lo.device)
        lay_lb = torch.cat([lay_lb, pad], dim=1).contiguous()
        lay_ub = torch.cat([lay_ub, pad], dim=1).contiguous()
    d = None
    if dead is not None:
        d = _c(dead, torch.uint8, (R, be.n_hidden), "dead")
    if R:
        ext().crown(_net(be), be.flat.data_ptr(), lo.data_ptr(), hi.data_ptr(), _ptr(d), R,
                    res.out_lb.data_ptr(), res.out_ub.data_ptr(), res.Lc.data_ptr(), res.L0.data_ptr(),
                    res.Le.data_ptr(), res.Uc.data_ptr(), res.U0.data_ptr(), res.Ue.data_ptr(),
                    lay_lb.data_ptr(), lay_ub.data_ptr(), _stream(lo.device))
    return res


# ------------------------------------------------------------------------------------------------
def refine(be, lo: torch.Tensor, hi: torch.Tensor, res: ref.BoundResult, dead: Optional[torch.Tensor] = None,
           phase: Optional[torch.Tensor] = None):
    """Back-substituted hidden-layer bounds (csrc/refine.hip) tightening ``res.layer_lb/ub`` in place
    (ref.crown_refine): ``res`` must come from :func:`bounds` with mode='symbolic' and
    keep_layers=True on the same rows.  Networks the kernel cannot hold keep the forward bounds.
    ``phase`` [R, n_hidden] int8 (ReLU-phase rows: +1 active / -1 inactive fixed, 0 free): the
    bounds hold on the region where the fixed phases hold, and ``res.infeasible`` [R] also marks rows
    whose refined bounds contradict a fixed phase (empty region)."""
    R, n0 = lo.shape
    if res.lay_lb_full is None:
        raise ValueError("refine needs symbolic bounds with keep_layers=True (HIP layout)")
    lo = _c(lo, torch.float32, (R, n0), "lo")
    hi = _c(hi, torch.float32, (R, n0), "hi")
    d = None
    if dead is not None:
        d = _c(dead, torch.uint8, (R, be.n_hidden), "dead")
    ph = _c(phase, torch.int8, (R, be.n_hidden), "phase") if phase is not None else None
    infeas = torch.zeros(R, dtype=torch.uint8, device=lo.device) if phase is not None else None
    if R:
        ext().refine(_net(be), be.flat.data_ptr(), lo.data_ptr(), hi.data_ptr(), _ptr(d), R,
                     res.lay_lb_full.data_ptr(), res.lay_ub_full.data_ptr(), _stream(lo.device), _ptr(ph),
                     _ptr(infeas))
    if infeas is not None:
        res.infeasible = infeas.bool() if res.infeasible is None else (res.infeasible | infeas.bool())
    Nh = be.n_hidden
    if Nh:
        res.dead = res.lay_ub_full[:, :Nh] <= 0
        res.dead_u8 = res.dead.to(torch.uint8)
        res.active = res.lay_lb_full[:, :Nh] >= 0
    return res


# ------------------------------------------------------------------------------------------------
def backward_bounds(be, lo: torch.Tensor, hi: torch.Tensor, dead: Optional[torch.Tensor] = None,
                    keep_layers: bool = True) -> Optional[ref.BoundResult]:
    """Every neuron's bounds and the logit's forms by back-substitution alone (csrc/refine.hip mode
    FULL, ref.backward_bounds).  ``None`` when the network does not fit the kernel."""
    R, n0 = lo.shape
    dev = lo.device
    lo = _c(lo, torch.float32, (R, n0), "lo")
    hi = _c(hi, torch.float32, (R, n0), "hi")
    f32 = dict(dtype=torch.float32, device=dev)
    res = ref.BoundResult(out_lb=torch.empty(R, **f32), out_ub=torch.empty(R, **f32),
                          Lc=torch.empty(R, n0, **f32), L0=torch.empty(R, **f32), Le=torch.empty(R, **f32),
                          Uc=torch.empty(R, n0, **f32), U0=torch.empty(R, **f32), Ue=torch.empty(R, **f32))
    N = be.mlp.n_neurons
    lay_lb = torch.empty(R, N, **f32) if keep_layers else None
    lay_ub = torch.empty(R, N, **f32) if keep_layers else None
    d = None
    if dead is not None:
        d = _c(dead, torch.uint8, (R, be.n_hidden), "dead")
    if R:
        rc = ext().backward_bounds(_net(be), be.flat.data_ptr(), lo.data_ptr(), hi.data_ptr(), _ptr(d), R,
                                   res.out_lb.data_ptr(), res.out_ub.data_ptr(), res.Lc.data_ptr(), res.L0.data_ptr(),
                                   res.Le.data_ptr(), res.Uc.data_ptr(), res.U0.data_ptr(), res.Ue.data_ptr(),
                                   _ptr(lay_lb), _ptr(lay_ub), _stream(dev))
        if rc == -1:
            return None
    if keep_layers:
        widths = be.mlp.widths
        offs = [0]
        for w in widths:
            offs.append(offs[-1] + w)
        res.layer_lb = [lay_lb[:, offs[i]:offs[i + 1]] for i in range(len(widths))]
        res.layer_ub = [lay_ub[:, offs[i]:offs[i + 1]] for i in range(len(widths))]
        res.lay_lb_full, res.lay_ub_full = lay_lb, lay_ub
        Nh = be.n_hidden
        res.dead = lay_ub[:, :Nh] <= 0
        if d is not None:
            res.dead = res.dead | d.bool()
        res.active = (lay_lb[:, :Nh] >= 0) & ~res.dead
    return res


# ------------------------------------------------------------------------------------------------
def crown_phase(be, lo: torch.Tensor, hi: torch.Tensor, res: ref.BoundResult, phase: Optional[torch.Tensor] = None):
    """ReLU-phase backward bounds (csrc/relu.hip: fa_crown_phase_kernel) on rows bounded by
    :func:`bounds` (symbolic, keep_layers, same ``phase``).  Refines ``res`` (logit bounds, forms)
    in place like ref.crown_phase + the caller's intersection, and returns
    (ref.PhaseCrown, None) -- the kernel writes the better input forms into ``res`` directly."""
    R, n0 = lo.shape
    dev = lo.device
    lo = _c(lo, torch.float32, (R, n0), "lo")
    hi = _c(hi, torch.float32, (R, n0), "hi")
    if res.lay_lb_full is None:
        raise ValueError("crown_phase needs bounds(..., keep_layers=True) from the HIP path")
    ph = _c(phase, torch.int8, (R, be.n_hidden), "phase") if phase is not None else None
    split = torch.full((R, 2), -1, dtype=torch.int32, device=dev)
    score = torch.zeros(R, 2, dtype=torch.float32, device=dev)
    low = torch.zeros(R, 2, dtype=torch.float32, device=dev)
    infeas = res.infeasible.to(torch.uint8).contiguous() if res.infeasible is not None else None
    if R:
        ext().crown_phase(_net(be), be.flat.data_ptr(), lo.data_ptr(), hi.data_ptr(), R, _ptr(ph),
                          res.lay_lb_full.data_ptr(), res.lay_ub_full.data_ptr(), _ptr(infeas),
                          res.out_lb.data_ptr(), res.out_ub.data_ptr(), res.Lc.data_ptr(), res.L0.data_ptr(),
                          res.Le.data_ptr(), res.Uc.data_ptr(), res.U0.data_ptr(), res.Ue.data_ptr(),
                          split.data_ptr(), score.data_ptr(), low.data_ptr(), _stream(dev))
    return ref.PhaseCrown(low=low, split=split.long(), score=score), None


# ------------------------------------------------------------------------------------------------
def pair_certify(be, res_x, res_xp, xlo, xhi, xplo, xphi, pairs, values, pa, shared, relaxed) -> ref.PairDecision:
    Nn, n0 = xlo.shape
    dev = xlo.device
    V = values.shape[0]
    Pp = pairs.shape[0]
    norient = 2 if relaxed else 1
    f32 = dict(dtype=torch.float32, device=dev)
    xlo = _c(xlo, torch.float32, (Nn, n0), "xlo")
    xhi = _c(xhi, torch.float32, (Nn, n0), "xhi")
    xplo = _c(xplo, torch.float32, (Nn, n0), "xplo")
    xphi = _c(xphi, torch.float32, (Nn, n0), "xphi")
    for r in (res_x, res_xp):
        if r.Lc is None or tuple(r.Lc.shape) != (Nn * V, n0):
            raise ValueError("pair_certify needs symbolic forms for Nn*V rows")
    pairs_c = _c(pairs, torch.int64, (Pp, 2), "pairs")
    values_c = _c(values, torch.int64, None, "values")
    sh = _c(shared, torch.uint8, (n0,), "shared")
    Q = Pp * norient
    gmin = torch.empty(Nn, Q, **f32)
    tstar = torch.empty(Nn, Q, **f32)
    open_ = torch.empty(Nn, dtype=torch.uint8, device=dev)
    score = torch.empty(Nn, **f32)
    split = torch.empty(Nn, dtype=torch.int64, device=dev)
    cx = torch.empty(Nn, n0, **f32)
    cxp = torch.empty(Nn, n0, **f32)
    cv = torch.empty(Nn, dtype=torch.int64, device=dev)
    co = torch.empty(Nn, dtype=torch.int64, device=dev)
    fx = [res_x.Lc, res_x.L0, res_x.Le, res_x.Uc, res_x.U0, res_x.Ue, res_x.out_lb, res_x.out_ub]
    fxp = [res_xp.Lc, res_xp.L0, res_xp.Le, res_xp.Uc, res_xp.U0, res_xp.Ue, res_xp.out_lb, res_xp.out_ub]
    fx = [_c(t, torch.float32) for t in fx]
    fxp = [_c(t, torch.float32) for t in fxp]
    scores = torch.empty(Nn, 2 * n0, **f32)
    leaf = torch.empty(Nn, dtype=torch.uint8, device=dev)
    if Nn:
        ext().certify(Nn, n0, V, Pp, norient, [t.data_ptr() for t in fx], [t.data_ptr() for t in fxp],
                      xlo.data_ptr(), xhi.data_ptr(), xplo.data_ptr(), xphi.data_ptr(), pairs_c.data_ptr(),
                      values_c.data_ptr(), [int(i) for i in pa.tolist()], [], 0.0, sh.data_ptr(), be.unit,
                      ref.gamma(2 * n0 + 4, be.unit), gmin.data_ptr(), tstar.data_ptr(), open_.data_ptr(),
                      score.data_ptr(), split.data_ptr(), cx.data_ptr(), cxp.data_ptr(), cv.data_ptr(),
                      co.data_ptr(), scores.data_ptr(), leaf.data_ptr(), _stream(dev))
    return ref.PairDecision(open_=open_.bool(), score=score, split_dim=split, cand_x=cx, cand_xp=cxp,
                            cand_v=cv, cand_orient=co)


# ------------------------------------------------------------------------------------------------
def _parse_sim_blocks(v: Optional[str]) -> int:
    if v is None or v.strip() == "":
        return 0
    try:
        n = int(v)
    except ValueError:
        raise ValueError(f"FAIRIFY_SIM_BLOCKS={v!r}: expected a non-negative integer") from None
    if n < 0:
        raise ValueError(f"FAIRIFY_SIM_BLOCKS={v!r}: expected a non-negative integer")
    return n


# parsed once at import (a bad value fails here, not inside a worker thread mid-run); tests that
# change the variable at run time set _SIM_BLOCKS_ENV = "dynamic" to re-read it per call
_SIM_BLOCKS = _parse_sim_blocks(os.environ.get("FAIRIFY_SIM_BLOCKS"))
_SIM_BLOCKS_ENV: Optional[str] = None


def _sim_split(P: int, n_samples: int) -> int:
    """Workgroups per partition for ``fa_sim_kernel``: with ``FAIRIFY_SIM_BLOCKS=B`` a short list
    of partitions with a large sample budget (the residual falsifier on a per-rank residue) is
    spread over about B workgroups instead of one per partition walking its 64-sample tiles
    serially.  Results are bit-identical either way (tests/test_kernels_gpu.py).  Off by default:
    with 8 concurrent host streams the extra blocks only contend with the other streams' bound
    kernels (A/B in profiles/r1_sim_split_ab.md)."""
    target = _SIM_BLOCKS if _SIM_BLOCKS_ENV is None else _parse_sim_blocks(os.environ.get("FAIRIFY_SIM_BLOCKS"))
    if not P or target <= P:
        return 1
    tiles = (n_samples + 63) // 64
    return max(1, min(tiles, -(-target // P)))


def simulate(be, q, lo, hi, pids, n_samples, seed, values, pairs, bisect_pairs, bisect_steps, return_z0=False):
    from ..engine.sim import SimResult, boundary_walk

    P, n0 = lo.shape
    dev = lo.device
    lo_c = _c(lo, torch.float32, (P, n0), "lo")
    hi_c = _c(hi, torch.float32, (P, n0), "hi")
    pids_c = _c(pids, torch.int64, (P,), "pids")
    V = values.shape[0]
    Pp = pairs.shape[0]
    values_c = _c(values, torch.int64, None, "values")
    pairs_c = _c(pairs, torch.int64, (Pp, 2), "pairs")
    split = _sim_split(P, n_samples)
    counts = (torch.zeros if split > 1 else torch.empty)(P, be.mlp.n_neurons, dtype=torch.int32, device=dev)
    keys = torch.full((P,), 0x7FFFFFFF, dtype=torch.int32, device=dev) if split > 1 else None
    found = torch.zeros(P, dtype=torch.uint8, device=dev)
    wx = torch.zeros(P, n0, dtype=torch.float32, device=dev)
    wxp = torch.zeros(P, n0, dtype=torch.float32, device=dev)
    z0 = torch.empty(P, n_samples, dtype=torch.float32, device=dev) if (bisect_pairs and bisect_steps) else None
    if P and n_samples:
        ext().sim(_net(be), be.flat.data_ptr(), lo_c.data_ptr(), hi_c.data_ptr(), pids_c.data_ptr(), P, n_samples,
                  int(seed) & 0xFFFFFFFF, V, list(q.pa_idx), values_c.data_ptr(), Pp, pairs_c.data_ptr(),
                  list(q.ra_idx) if q.relaxed else [], int(q.tau), counts.data_ptr(), found.data_ptr(),
                  wx.data_ptr(), wxp.data_ptr(), _ptr(z0), _ptr(keys), split, _stream(dev))
    res = SimResult(counts=counts, found=found.bool(), wit_x=wx, wit_xp=wxp)
    if z0 is not None:
        boundary_walk(be, q, lo_c, hi_c, pids_c, n_samples, seed, values_c, pairs_c, res, z0, bisect_pairs,
                      bisect_steps)
    return res


def ascent(be, q, lo, hi, x0, f0, q0, iters, values, pairs, free_dims):
    """Lattice coordinate ascent of the residual falsifier in one launch (``fa_ascent_kernel``).

    ``x0`` [P, K, n0] start points, ``f0`` [P, K] their margins, ``q0`` [P, K] pair indices.
    Returns ``(found [P] bool, wit_x [P, n0], wit_xp [P, n0])``, or ``None`` when one partition's
    candidate rows do not fit in LDS (the caller then runs the PyTorch loop)."""
    P, K, n0 = x0.shape
    dev = x0.device
    lo_c = _c(lo, torch.float32, (P, n0), "lo")
    hi_c = _c(hi, torch.float32, (P, n0), "hi")
    x0_c = _c(x0, torch.float32, (P, K, n0), "x0")
    f0_c = _c(f0, torch.float32, (P, K), "f0")
    q0_c = _c(q0, torch.int32, (P, K), "q0")
    V = values.shape[0]
    Pp = pairs.shape[0]
    values_c = _c(values, torch.int64, None, "values")
    pairs_c = _c(pairs, torch.int64, (Pp, 2), "pairs")
    found = torch.zeros(P, dtype=torch.uint8, device=dev)
    wx = torch.zeros(P, n0, dtype=torch.float32, device=dev)
    wxp = torch.zeros(P, n0, dtype=torch.float32, device=dev)
    if P == 0:
        return found.bool(), wx, wxp
    ok = ext().ascent(_net(be), be.flat.data_ptr(), lo_c.data_ptr(), hi_c.data_ptr(), x0_c.data_ptr(),
                      f0_c.data_ptr(), q0_c.data_ptr(), P, K, int(iters), V, list(q.pa_idx), values_c.data_ptr(),
                      Pp, pairs_c.data_ptr(), [int(d) for d in free_dims], found.data_ptr(), wx.data_ptr(),
                      wxp.data_ptr(), _stream(dev))
    if not ok:
        return None
    return found.bool(), wx, wxp


def falsify(be, q, lo, hi, pids, values, pairs, seed, n_samples, n_local, walk_k, walk_steps, k_starts, iters,
            free_dims, dseed: int = 0):
    """Fused residual falsifier (``csrc/falsify.hip``): heavy sampling, boundary walk, lattice
    coordinate ascent in one launch.  Relaxed queries: x' carries RA offsets in [-tau, tau] (hash
    stream ``dseed`` per sample, moved by the ascent), both orientations of every pair count.
    Returns ``(found [P] bool, wit_x [P, n0], wit_xp [P, n0], how [P] int8)`` or ``None`` when the
    network shape is not supported by the kernel (the caller keeps the PyTorch path)."""
    P, n0 = lo.shape
    dev = lo.device
    lo_c = _c(lo, torch.float32, (P, n0), "lo")
    hi_c = _c(hi, torch.float32, (P, n0), "hi")
    pids_c = _c(pids, torch.int64, (P,), "pids")
    V = values.shape[0]
    Pp = pairs.shape[0]
    values_c = _c(values, torch.int64, None, "values")
    pairs_c = _c(pairs, torch.int64, (Pp, 2), "pairs")
    if values_c.numel() != V * len(q.pa_idx):
        raise ValueError("values: expected [V, n_pa]")
    found = torch.zeros(P, dtype=torch.uint8, device=dev)
    wx = torch.zeros(P, n0, dtype=torch.float32, device=dev)
    wxp = torch.zeros(P, n0, dtype=torch.float32, device=dev)
    how = torch.zeros(P, dtype=torch.int8, device=dev)
    if P == 0 or Pp == 0 or n_samples <= 0:
        return found.bool(), wx, wxp, how
    ok = ext().falsify(_net(be), be.flat.data_ptr(), lo_c.data_ptr(), hi_c.data_ptr(), pids_c.data_ptr(), P,
                       int(n_samples), int(n_local), int(seed) & 0xFFFFFFFF, V, list(q.pa_idx), values_c.data_ptr(),
                       Pp, pairs_c.data_ptr(), int(walk_k), int(walk_steps), int(k_starts), int(iters),
                       [int(d) for d in free_dims], found.data_ptr(), wx.data_ptr(), wxp.data_ptr(), how.data_ptr(),
                       _stream(dev), list(q.ra_idx) if q.relaxed else [], int(q.tau) if q.relaxed else 0,
                       int(dseed) & 0xFFFFFFFF)
    if not ok:
        return None
    return found.bool(), wx, wxp, how


# ------------------------------------------------------------------------------------------------
def prune_masks(be, counts: torch.Tensor, lay_ub: torch.Tensor, sym_dead: Optional[torch.Tensor]):
    """Sound-prune mask algebra of the pipeline's stage 2 in one launch (``csrc/prune.hip``).

    ``counts`` [P, N] int32 simulation activation counts, ``lay_ub`` [P, N] IBP upper bounds,
    ``sym_dead`` [P, N_hidden] uint8 symbolic stable-inactive flags (or None).  Returns
    ``(code [P, N] uint8, cnt [P, 3] int32)``: per neuron bit 0 candidate, 1 bound-dead, 2
    symbolic-dead, 3 merged sound dead, 4 symbolic candidate; per partition the B/S/ST dead
    counts."""
    P, N = counts.shape
    dev = counts.device
    counts_c = _c(counts, torch.int32, (P, be.mlp.n_neurons), "counts")
    ub_c = _c(lay_ub, torch.float32, (P, N), "lay_ub")
    sd = None
    if sym_dead is not None:
        sd = _c(sym_dead, torch.uint8, (P, be.n_hidden), "sym_dead")
    code = torch.empty(P, N, dtype=torch.uint8, device=dev)
    cnt = torch.empty(P, 3, dtype=torch.int32, device=dev)
    if P:
        ext().prune_masks(_net(be), P, counts_c.data_ptr(), ub_c.data_ptr(), N, _ptr(sd), code.data_ptr(),
                          cnt.data_ptr(), _stream(dev))
    return code, cnt


PM_CAND, PM_B, PM_S, PM_ST, PM_SCAND = 1, 2, 4, 8, 16


def heuristic(be, rows: torch.Tensor, lay_lb: torch.Tensor, lay_ub: torch.Tensor, code: torch.Tensor, perc: float):
    """The reference's heuristic pruning (utils/prune.py:862-939) for partitions ``rows`` of the
    stage-2 arrays, one wave per partition (K5).  Returns ``(new [Pu, N] uint8, merged [Pu, N]
    uint8, cnt [Pu, 2] int32 = (#new, #merged))``."""
    Pu = rows.shape[0]
    P, N = lay_ub.shape
    dev = lay_ub.device
    rows_c = _c(rows, torch.int64, (Pu,), "rows")
    lb_c = _c(lay_lb, torch.float32, (P, N), "lay_lb")
    ub_c = _c(lay_ub, torch.float32, (P, N), "lay_ub")
    code_c = _c(code, torch.uint8, (P, N), "code")
    hnew = torch.empty(Pu, N, dtype=torch.uint8, device=dev)
    hmerged = torch.empty(Pu, N, dtype=torch.uint8, device=dev)
    cnt = torch.empty(Pu, 2, dtype=torch.int32, device=dev)
    if Pu:
        ext().heuristic(_net(be), Pu, rows_c.data_ptr(), lb_c.data_ptr(), ub_c.data_ptr(), N, code_c.data_ptr(),
                        50.0 / 100.0, float(perc) / 100.0, (100.0 - float(perc)) / 100.0, hnew.data_ptr(),
                        hmerged.data_ptr(), cnt.data_ptr(), _stream(dev))
    return hnew, hmerged, cnt


def agree(be, rows: torch.Tensor, lo: torch.Tensor, hi: torch.Tensor, pids: torch.Tensor, dead: torch.Tensor,
          n_samples: int, seed: int):
    """Pruned-acc / Pruned-F1 counts: per partition ``rows[k]``, over its ``n_samples``
    simulation points, (points where the full network and the network with ``dead[k]``
    [N_hidden] forced to zero agree in sign, points positive for both, points positive only for
    the pruned network).  Returns int32 [Pm, 3] or ``None`` (shape unsupported: caller keeps
    PyTorch)."""
    Pm = rows.shape[0]
    P, n0 = lo.shape
    dev = lo.device
    rows_c = _c(rows, torch.int64, (Pm,), "rows")
    lo_c = _c(lo, torch.float32, (P, n0), "lo")
    hi_c = _c(hi, torch.float32, (P, n0), "hi")
    pids_c = _c(pids, torch.int64, (P,), "pids")
    dead_c = _c(dead, torch.uint8, (Pm, be.n_hidden), "dead")
    out = torch.zeros(Pm, 3, dtype=torch.int32, device=dev)
    if Pm == 0:
        return out
    ok = ext().agree(_net(be), be.flat.data_ptr(), Pm, rows_c.data_ptr(), lo_c.data_ptr(), hi_c.data_ptr(),
                     pids_c.data_ptr(), dead_c.data_ptr(), int(n_samples), int(seed) & 0xFFFFFFFF, out.data_ptr(),
                     _stream(dev))
    return out if ok else None


# ------------------------------------------------------------------------------------------------
def _beta_wt(be) -> torch.Tensor:
    """Per layer W_l transposed ([out][in] row-major) at the flat offsets of W_l (csrc/beta.hip's
    backward-operand copy), cached on the backend."""
    wt = getattr(be, "_beta_wt", None)
    if wt is None:
        import numpy as np

        with _LAZY_LOCK:          # built once: native runtimes keep its device pointer for the backend's life
            wt = getattr(be, "_beta_wt", None)
            if wt is None:
                parts = []
                for w, b in zip(be.mlp.weights, be.mlp.biases):
                    parts += [np.ascontiguousarray(np.asarray(w, np.float32).T).reshape(-1),
                              np.zeros(np.size(b), np.float32)]
                wt = torch.from_numpy(np.concatenate(parts)).to(be.device)
                if wt.is_cuda:
                    torch.cuda.current_stream(wt.device).synchronize()   # complete for every stream
                be._beta_wt = wt
    return wt


def beta_level(be, lo, hi, pa, va, vb, LBA, UBA, LBB, UBB, phA, phB, alA, alB, beA, beB, t, iters, lr_a, lr_b, lr_t,
               decay=1.0, lookahead=0, beta_pos=True, rx=None, stall=True, pgap=False, osg=None, feas_iters=0,
               feas_lr=None):
    """One beta-CROWN BaB level on the device (``fa_beta_kernel``, csrc/beta.hip): the rows'
    (alpha, beta, t) are optimised IN PLACE (kept at the best iterate) and their rigorous fp64
    bounds, branching decisions, concretising vertices and child multipliers returned
    (:class:`ops.beta.BetaLevel`)."""
    from . import beta as B

    R, n0 = lo.shape
    NH = be.n_hidden
    dev = lo.device
    npa = len(pa)
    if list(pa) != sorted(pa):
        raise ValueError("beta_level: PA dims must be increasing")
    f32 = dict(dtype=torch.float32, device=dev)
    lo_c = _c(lo, torch.float32, (R, n0), "lo")
    hi_c = _c(hi, torch.float32, (R, n0), "hi")
    va_c = _c(va, torch.float32, (R, npa), "va")
    vb_c = _c(vb, torch.float32, (R, npa), "vb")
    bnd = [_c(x, torch.float32, (R, NH), nm) for x, nm in ((LBA, "LBA"), (UBA, "UBA"), (LBB, "LBB"), (UBB, "UBB"))]
    pA = _c(phA, torch.int8, (R, NH), "phA")
    pB = _c(phB, torch.int8, (R, NH), "phB")
    for x, nm in ((alA, "alA"), (alB, "alB"), (beA, "beA"), (beB, "beB")):
        if tuple(x.shape) != (R, NH) or x.dtype != torch.float32:
            raise ValueError(f"{nm}: expected float32 [{R}, {NH}]")
    if tuple(t.shape) != (R,) or t.dtype != torch.float32 or not t.is_contiguous():
        raise ValueError("t: expected contiguous float32 [R]")
    par = torch.stack([alA, alB, beA, beB], 1).contiguous()          # [R, 4, NH]
    scratch = torch.empty(R, 16 if feas_iters > 0 else 12, NH, **f32)
    bound = torch.empty(R, dtype=torch.float64, device=dev)
    split = torch.empty(R, dtype=torch.int32, device=dev)
    xstar = torch.empty(R, n0, **f32)
    binit = torch.empty(R, 2, **f32)
    xpstar = torch.empty(R, n0, **f32)
    ramask, plo_c, phi_c, gt, tau = 0, None, None, None, 0.0
    if rx is not None:          # relaxed: copy B's RA dims over [plo, phi]
        for d in torch.nonzero(rx[0].cpu()).flatten().tolist():
            ramask |= 1 << int(d)
        plo_c = _c(rx[1], torch.float32, (R, n0), "plo")
        phi_c = _c(rx[2], torch.float32, (R, n0), "phi")
        if len(rx) > 3 and rx[4] is not None:       # the tau tie's multipliers (in / out)
            tau = float(rx[3])
            for x, nm in ((rx[4], "gP"), (rx[5], "gM")):
                if tuple(x.shape) != (R, n0) or x.dtype != torch.float32:
                    raise ValueError(f"{nm}: expected float32 [{R}, {n0}]")
            gt = torch.stack([rx[4], rx[5]], 1).contiguous()       # [R, 2, n0]
    osg_c = None if osg is None else _c(osg, torch.int8, (R,), "osg")
    if R:
        def launch(n_it, flags, lra, lrb, lrt):
            return ext().beta_level(_net(be), be.flat.data_ptr(), _beta_wt(be).data_ptr(), R, [int(d) for d in pa],
                                    lo_c.data_ptr(), hi_c.data_ptr(), va_c.data_ptr(), vb_c.data_ptr(),
                                    *[x.data_ptr() for x in bnd], pA.data_ptr(), pB.data_ptr(), par.data_ptr(),
                                    t.data_ptr(), scratch.data_ptr(), int(n_it), float(lra), float(lrb), float(lrt),
                                    float(decay), int(lookahead), int(bool(beta_pos)), flags, bound.data_ptr(),
                                    split.data_ptr(), xstar.data_ptr(), binit.data_ptr(), int(ramask), _ptr(plo_c),
                                    _ptr(phi_c), xpstar.data_ptr(), _ptr(gt), float(tau), _ptr(osg_c), _stream(dev))

        rc = launch(iters, int(bool(stall)) | (int(pgap) << 1), lr_a, lr_b, lr_t)
        if rc == 0 and feas_iters > 0:
            # the infeasibility pass (bit 3) on the nodes left open: only their bounds can change
            rc = launch(feas_iters, 8, *(feas_lr or (lr_a, lr_b, lr_t)))
        if rc != 0:
            raise RuntimeError(f"fa_beta_kernel launch failed ({rc}): network not supported by the beta kernel")
        if gt is not None:
            rx[4].copy_(gt[:, 0])
            rx[5].copy_(gt[:, 1])
        alA.copy_(par[:, 0])
        alB.copy_(par[:, 1])
        beA.copy_(par[:, 2])
        beB.copy_(par[:, 3])
    return B.BetaLevel(bound=bound, split=split.long(), xstar=xstar, binit=binit, xpstar=xpstar)
