"""Per-model compute backend: weights resident on the device + the hot ops.

One ``Backend`` is created per (model, device).  Weights are uploaded once (≤ 90 KB fp32 for
the largest zoo model) and, for the HIP path, packed into the flat layout the kernels read
(``[W_0 | b_0 | W_1 | b_1 | ...]`` fp32, Keras ``[in, out]`` row-major).  Every method takes
and returns device tensors; on CUDA/ROCm devices the HIP kernels run, on CPU the PyTorch
reference in :mod:`fairify_amd.ops.reference`.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch

from ..models.mlp import MLP
from . import reference as ref
from . import use_hip


def mfma_weight_block(weights, biases) -> np.ndarray:
    """Weights in MFMA operand order for the register-resident kernels (csrc/symbolic.hip,
    csrc/points.hip): per layer [jt][t][lane][i] = W[16t + 4(lane>>4) + i][16jt + (lane&15)]
    (zero padded to 16-neuron tiles), then every layer's bias; total padded to 4 floats."""
    parts = []
    lane = np.arange(64)
    for W in weights:
        n_in, n_out = W.shape
        tin, tout = (n_in + 15) // 16, (n_out + 15) // 16
        Wp = np.zeros((16 * tin, 16 * tout), np.float32)
        Wp[:n_in, :n_out] = W
        jt, t, ln, i = np.meshgrid(np.arange(tout), np.arange(tin), lane, np.arange(4), indexing="ij")
        parts.append(Wp[16 * t + 4 * (ln >> 4) + i, 16 * jt + (ln & 15)].reshape(-1))
    parts += [np.asarray(b, np.float32).reshape(-1) for b in biases]
    out = np.concatenate(parts)
    return np.concatenate([out, np.zeros((-len(out)) % 4, np.float32)])


def mfma_back_block(weights) -> np.ndarray:
    """Weights in backward (transposed) MFMA operand order, read from global memory by
    csrc/refine.hip when staging them would leave too little LDS for its per-row state: per layer
    [ot][t][lane][i] = W[16 ot + (lane&15)][16 t + 4(lane>>4) + i] (zero padded), ot over input
    tiles, t over output tiles -- the layout that kernel stages into LDS.  Must match
    ``Net::wback_off`` / ``wback_floats`` in csrc/bindings.cpp (appended last)."""
    parts = []
    lane = np.arange(64)
    for W in weights:
        n_in, n_out = W.shape
        tin, tout = (n_in + 15) // 16, (n_out + 15) // 16
        Wp = np.zeros((16 * tin, 16 * tout), np.float32)
        Wp[:n_in, :n_out] = W
        ot, t, ln, i = np.meshgrid(np.arange(tin), np.arange(tout), lane, np.arange(4), indexing="ij")
        parts.append(Wp[16 * ot + (ln & 15), 16 * t + 4 * (ln >> 4) + i].reshape(-1))
    return np.concatenate(parts)


def pack_groups(dims) -> int:
    """Boxes packed per 16-row MFMA tile by the symbolic kernel for narrow single-tile networks
    (csrc/symbolic.hip, ``PG``): inputs <= 16 and every hidden layer <= 8 wide.  Box g owns tile
    rows g*S .. g*S+S-1 with S = 16 / PG a multiple of 4, so every box's K terms fall into the
    MFMA's 4-wide K steps exactly as an unpacked box's do: a box's bounds are bitwise those of the
    unpacked kernel and never depend on which boxes share its tile (node order in the BaB pool
    follows device atomics).  Widest hidden layer <= 4 -> 4 boxes, <= 8 -> 2.  Must equal
    ``Net::pack_g`` in csrc/bindings.cpp."""
    dims = list(dims)
    L = len(dims) - 1
    if L < 2 or dims[0] > 16 or max(dims) > 16:
        return 1
    mh = max(dims[1:L])
    return 4 if mh <= 4 else (2 if mh <= 8 else 1)


def mfma_packed_block(weights, biases, G: int) -> np.ndarray:
    """Block-diagonal weights of G boxes per tile (narrow networks, csrc/symbolic.hip ``PG``), MFMA
    operand order [t][lane][i] = W[16t + 4(lane>>4) + i][lane&15] per tile, box stride S = 16 / G:

    * layer 0: G tiles, tile g = W_0 (n0 x w_1) at rows 0.., columns g*S.. (box g's inputs feed
      its own output rows);
    * layer l >= 1: one tile, W_l at rows g*S.., columns g*S.. for every box g;
    * then 16 bias floats per layer (b_l at g*S.. for every box g)."""
    lane = np.arange(64)
    t_, ln, i_ = np.meshgrid(np.arange(1), lane, np.arange(4), indexing="ij")
    S = 16 // G

    def tile(M):
        return M[4 * (ln >> 4) + i_, ln & 15].reshape(-1)

    parts = []
    W0 = np.asarray(weights[0], np.float32)
    n0, w1 = W0.shape
    for g in range(G):
        M = np.zeros((16, 16), np.float32)
        M[:n0, g * S:g * S + w1] = W0
        parts.append(tile(M))
    for W in weights[1:]:
        W = np.asarray(W, np.float32)
        M = np.zeros((16, 16), np.float32)
        for g in range(G):
            M[g * S:g * S + W.shape[0], g * S:g * S + W.shape[1]] = W
        parts.append(tile(M))
    for b in biases:
        pb = np.zeros(16, np.float32)
        b = np.asarray(b, np.float32).reshape(-1)
        for g in range(G):
            pb[g * S:g * S + b.size] = b
        parts.append(pb)
    return np.concatenate(parts)


class Backend:
    def __init__(self, mlp: MLP, device="cpu", dtype=torch.float32):
        self.mlp = mlp
        self.device = torch.device(device)
        self.dtype = dtype
        self.ws = [torch.from_numpy(w).to(self.device, dtype) for w in mlp.weights]
        self.bs = [torch.from_numpy(b).to(self.device, dtype) for b in mlp.biases]
        self.widths = mlp.widths
        self.n0 = mlp.n_in
        self.n_hidden = int(sum(mlp.hidden))
        probe = torch.empty(0, device=self.device)
        self.hip = use_hip(probe) and dtype == torch.float32
        if self.hip:
            from . import ext

            # dynamic-LDS limits of every >64 KB kernel, once per process, before any host thread
            # launches (csrc/common.h registry; no launch path sets a function attribute)
            rc = ext().prepare_lds()
            if rc != 0:
                raise RuntimeError(f"fa_lds_prepare failed ({rc})")
            flat = np.concatenate([np.concatenate([w.reshape(-1), b]) for w, b in zip(mlp.weights, mlp.biases)])
            flat = np.concatenate([flat.astype(np.float32), np.zeros((-len(flat)) % 4, np.float32),
                                   mfma_weight_block(mlp.weights, mlp.biases)])
            G = pack_groups([mlp.n_in] + mlp.widths)
            if G > 1:
                flat = np.concatenate([flat, mfma_packed_block(mlp.weights, mlp.biases, G)])
            flat = np.concatenate([flat, mfma_back_block(mlp.weights)])
            self.flat = torch.from_numpy(flat).to(self.device)
            dims = [mlp.n_in] + mlp.widths
            self.dims = torch.tensor(dims, dtype=torch.int32)
        self.unit = ref.FP32_UNIT if dtype == torch.float32 else ref.FP64_UNIT

    # ----------------------------------------------------------------------------- forward
    def forward(self, x: torch.Tensor, dead: Optional[torch.Tensor] = None) -> torch.Tensor:
        x = x.to(self.dtype)
        if self.hip:
            from . import hip

            return hip.forward(self, x, dead)
        return ref.forward(self.ws, self.bs, x, dead)

    def forward_error(self, x: torch.Tensor) -> torch.Tensor:
        return ref.forward_error_bound(self.ws, self.bs, x.to(self.dtype), self.unit)

    def activation_counts(self, x: torch.Tensor) -> torch.Tensor:
        """x [B, S, n0] -> [B, N] non-zero counts per neuron (all layers)."""
        if self.hip:
            from . import hip

            return hip.activation_counts(self, x.to(self.dtype))
        return ref.activation_counts(self.ws, self.bs, x.to(self.dtype))

    # ----------------------------------------------------------------------------- bounds
    def bounds(self, lo: torch.Tensor, hi: torch.Tensor, mode: str = "symbolic",
               dead: Optional[torch.Tensor] = None, keep_layers: bool = False, fold=(),
               crown: bool = False, phase: Optional[torch.Tensor] = None, refine: bool = False) -> ref.BoundResult:
        """``fold``: dims degenerate (lo == hi) in every row — a HIP-kernel layout hint only.
        ``crown``: refine the logit forms/bounds with the backward pass (symbolic mode only).
        ``refine`` (with ``crown``): first tighten the hidden layers' bounds by back-substitution
        (ref.crown_refine / csrc/refine.hip), then run the backward output pass on them.
        ``phase``: [R, N_hidden] int8 ReLU phases of the rows' branch regions (-1 / 0 / +1,
        ref.bounds); the result's ``infeasible`` flags rows whose region is empty."""
        lo = lo.to(self.dtype)
        hi = hi.to(self.dtype)
        if mode == "backward":
            # every bound by back-substitution alone (ref.backward_bounds / csrc/refine.hip FULL)
            if self.hip:
                from . import hip

                r = hip.backward_bounds(self, lo, hi, dead)
                if r is not None:
                    return r
                mode, crown, refine = "symbolic", True, True
            else:
                return ref.backward_bounds(self.ws, self.bs, lo, hi, dead, unit=self.unit)
        crown = crown and mode == "symbolic"
        if self.hip:
            from . import hip

            r = hip.bounds(self, lo, hi, mode=mode, dead=dead, keep_layers=keep_layers or crown, fold=fold,
                           phase=phase)
            if crown and refine:
                r = hip.refine(self, lo, hi, r, dead)
            return hip.crown(self, lo, hi, r, dead) if crown else r
        r = ref.bounds(self.ws, self.bs, lo, hi, mode=mode, dead=dead, unit=self.unit,
                       keep_layers=keep_layers or crown, phase=phase)
        if crown and refine:
            r = ref.crown_refine(self.ws, self.bs, lo, hi, r, dead, unit=self.unit)
        return ref.crown_output(self.ws, self.bs, lo, hi, r, dead, unit=self.unit) if crown else r

    def crown_phase(self, lo: torch.Tensor, hi: torch.Tensor, res: ref.BoundResult,
                    phase: Optional[torch.Tensor] = None):
        """Backward bounds of the ReLU-phase search concretised at every layer (ref.crown_phase)."""
        lo = lo.to(self.dtype)
        hi = hi.to(self.dtype)
        if self.hip:
            from . import hip

            return hip.crown_phase(self, lo, hi, res, phase)
        return ref.crown_phase(self.ws, self.bs, lo, hi, res, phase, unit=self.unit)

    def point_bounds(self, x: torch.Tensor, dead: Optional[torch.Tensor] = None):
        """Rigorous [lb, ub] of the logit at points x [R, n0] (candidate-pair screening)."""
        x = x.to(self.dtype)
        if self.hip:
            from . import hip

            return hip.point_bounds(self, x, dead)
        return ref.point_bounds(self.ws, self.bs, x, dead, unit=self.unit)

    def phase_layer_bounds(self, lo: torch.Tensor, hi: torch.Tensor, phase: torch.Tensor):
        """Rigorous pre-activation bounds [R, NH] of every hidden neuron over each row's box AND its
        phase region (forward symbolic with the phases fixed, then back-substituted refinement:
        csrc/refine.hip with ``phase_in``), and the rows whose region those bounds prove empty.
        CPU: the reference refines without the phases (valid, looser)."""
        NH = self.n_hidden
        lo = lo.to(self.dtype)
        hi = hi.to(self.dtype)
        if self.hip:
            from . import hip

            r = hip.bounds(self, lo, hi, mode="symbolic", keep_layers=True, phase=phase)
            r = hip.refine(self, lo, hi, r, phase=phase)
            return r.lay_lb_full[:, :NH], r.lay_ub_full[:, :NH], r.infeasible
        r = ref.bounds(self.ws, self.bs, lo, hi, mode="symbolic", unit=self.unit, keep_layers=True, phase=phase)
        inf = r.infeasible
        r = ref.crown_refine(self.ws, self.bs, lo, hi, r, unit=self.unit)
        lb = torch.cat([t for t in r.layer_lb], 1)[:, :NH]
        ub = torch.cat([t for t in r.layer_ub], 1)[:, :NH]
        return lb, ub, inf

    def beta_level(self, lo, hi, pa, va, vb, LBA, UBA, LBB, UBB, phA, phB, alA, alB, beA, beB, t, iters: int,
                   lr_a: float, lr_b: float, lr_t: float, decay: float = 1.0, lookahead: int = 0,
                   beta_pos: bool = True, rx=None, stall: bool = True, pgap: int = 0, osg=None,
                   feas_iters: int = 0, feas_lr=None):
        """One beta-CROWN BaB level (ops/beta.py): optimises the rows' (alpha, beta, t) IN PLACE and
        returns their rigorous fp64 bounds, branching decisions and concretising vertices."""
        if self.hip:
            from . import hip

            return hip.beta_level(self, lo, hi, pa, va, vb, LBA, UBA, LBB, UBB, phA, phB, alA, alB, beA, beB, t,
                                  iters, lr_a, lr_b, lr_t, decay, lookahead, beta_pos, rx, stall, pgap, osg,
                                  feas_iters, feas_lr)
        from . import beta

        return beta.level_ref([w.float() for w in self.ws], [b.float() for b in self.bs], self.widths[:-1], lo, hi,
                              pa, va, vb, LBA, UBA, LBB, UBB, phA, phB, alA, alB, beA, beB, t, iters, lr_a, lr_b,
                              lr_t, decay, lookahead, beta_pos, rx, stall, pgap, osg, feas_iters, feas_lr)

    # ----------------------------------------------------------------------------- BaB node test
    def pair_certify(self, res_x, res_xp, xlo, xhi, xplo, xphi, pairs, values, pa, shared, relaxed):
        if self.hip:
            from . import hip

            return hip.pair_certify(self, res_x, res_xp, xlo, xhi, xplo, xphi, pairs, values, pa, shared, relaxed)
        return ref.pair_certify(res_x, res_xp, xlo.to(self.dtype), xhi.to(self.dtype), xplo.to(self.dtype),
                                xphi.to(self.dtype), pairs, values, pa, shared, relaxed, unit=self.unit)
