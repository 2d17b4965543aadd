"""SMT-LIB2 encoding of the partition fairness query (host side).

Re-creates what the reference builds with the Z3 Python API for one partition
(src/AC/Verify-AC.py:127-158, src/GC/Verify-GC.py:124-158):

* integer variables ``x0..x{n-1}`` and ``x_0..x_{n-1}`` (src/AC/Verify-AC.py:131-132);
* the network twice, ``y = N'(x)``, ``y' = N'(x')`` over the (sound-pruned) weights, in real
  arithmetic on ``to_real`` of the inputs with ReLU ``ite(v >= 0, v, 0)``
  (``z3_net`` in utils/*-Model-Functions.py, ``z3Relu`` utils/verif_utils.py:525-528);
* the domain constraints ``lo <= x_i <= hi`` for every i and ``lo <= x'_p <= hi`` for every
  protected attribute p (``in_const_domain_*`` utils/verif_utils.py:743-856);
* ``x_p != x'_p`` for p in PA, ``|x_r - x'_r| <= tau`` for r in RA (``in_const_diff_*``
  :859-907), ``x_a = x'_a`` otherwise (``in_const_*`` eq, :1065-1091);
* the sign flip ``(y < 0 and y' > 0) or (y > 0 and y' < 0)`` (src/AC/Verify-AC.py:155).

Differences (documented, deliberate): weights are written as the EXACT rationals of their fp32
values (the reference passes numpy floats through Z3's float conversion), intermediate neurons
are named with ``define-fun`` so the formula stays linear in size, and the soft timeout is an
``(set-option :timeout ms)`` line (``Solver.set("timeout", ...)``, src/AC/Verify-AC.py:147-150).
The fork's solver parameters (``random_seed=42, restart.max=100, phase_selection=0``,
src/AC/Verify-AC-experiment.py:163-165) are emitted as options when requested.

The host encoder consumes networks that the GPU already pruned (dead neurons removed,
:meth:`fairify_amd.models.mlp.MLP.prune`), exactly like the reference feeds ``pr_w, pr_b``.
"""
from __future__ import annotations

from dataclasses import dataclass
from fractions import Fraction
from typing import List, Optional, Sequence

import numpy as np

from ..models.mlp import MLP
from ..spec import ResolvedQuery


def rational(v: float) -> str:
    """Exact SMT-LIB real literal of a binary float (``(/ p q)`` or ``(- (/ p q))``)."""
    f = Fraction(float(v))
    p, q = abs(f.numerator), f.denominator
    body = f"{p}.0" if q == 1 else f"(/ {p}.0 {q}.0)"
    return f"(- {body})" if f < 0 else body


def _int(v: int) -> str:
    v = int(v)
    return str(v) if v >= 0 else f"(- {-v})"


def xname(i: int, prime: bool = False) -> str:
    return f"x_{i}" if prime else f"x{i}"


def _net_defs(mlp: MLP, prime: bool, tag: str) -> List[str]:
    """define-fun chain of the network on inputs x (or x'); returns lines, last one names the logit."""
    lines: List[str] = []
    n0 = mlp.n_in
    prev = [f"(to_real {xname(i, prime)})" for i in range(n0)]
    L = mlp.n_layers
    for l, (W, b) in enumerate(zip(mlp.weights, mlp.biases)):
        cur = []
        for j in range(W.shape[1]):
            terms = []
            for k in range(W.shape[0]):
                w = float(W[k, j])
                if w != 0.0:
                    terms.append(f"(* {rational(w)} {prev[k]})")
            terms.append(rational(float(b[j])))
            s = terms[0] if len(terms) == 1 else "(+ " + " ".join(terms) + ")"
            name = f"{tag}_l{l}_{j}"
            if l < L - 1:
                lines.append(f"(define-fun {name}_pre () Real {s})")
                lines.append(f"(define-fun {name} () Real (ite (>= {name}_pre 0.0) {name}_pre 0.0))")
            else:
                lines.append(f"(define-fun {name} () Real {s})")
            cur.append(name)
        prev = cur
    lines.append(f"(define-fun {tag} () Real {prev[0]})")
    return lines


@dataclass
class SMTQuery:
    text: str
    n: int

    def __str__(self) -> str:
        return self.text


def encode_partition(mlp: MLP, q: ResolvedQuery, lo: Sequence[int], hi: Sequence[int],
                     timeout_s: Optional[float] = None, fork_params: bool = False,
                     get_model: bool = True) -> SMTQuery:
    """SMT-LIB2 script deciding one partition box ``[lo, hi]`` for network ``mlp``."""
    n = q.n
    if mlp.n_in != n:
        raise ValueError(f"network has {mlp.n_in} inputs, domain has {n}")
    pa, ra = set(q.pa_idx), set(q.ra_idx) if q.relaxed else set()
    out = ["(set-option :produce-models true)"]
    if timeout_s is not None:
        out.append(f"(set-option :timeout {int(round(timeout_s * 1000))})")
    if fork_params:
        out += ["(set-option :random-seed 42)", "(set-option :smt.restart.max 100)",
                "(set-option :smt.phase_selection 0)"]
    for i in range(n):
        out.append(f"(declare-fun {xname(i)} () Int)")
    for i in range(n):
        out.append(f"(declare-fun {xname(i, True)} () Int)")
    out += _net_defs(mlp, False, "y")
    out += _net_defs(mlp, True, "yp")
    # domain (in_const_domain_*): every x_i, and x'_p for protected attributes
    for i in range(n):
        out.append(f"(assert (and (<= {_int(lo[i])} {xname(i)}) (<= {xname(i)} {_int(hi[i])})))")
    for p in sorted(pa):
        out.append(f"(assert (and (<= {_int(lo[p])} {xname(p, True)}) (<= {xname(p, True)} {_int(hi[p])})))")
    # fairness pre-condition
    for i in range(n):
        if i in pa:
            out.append(f"(assert (not (= {xname(i)} {xname(i, True)})))")
        elif i in ra:
            d = f"(- {xname(i)} {xname(i, True)})"
            out.append(f"(assert (and (<= {d} {_int(q.tau)}) (<= (- {d}) {_int(q.tau)})))")
        else:
            out.append(f"(assert (= {xname(i)} {xname(i, True)}))")
    # sign-flip post-condition (strict)
    out.append("(assert (or (and (< y 0.0) (> yp 0.0)) (and (> y 0.0) (< yp 0.0))))")
    out.append("(check-sat)")
    if get_model:
        out.append("(get-model)")
    return SMTQuery(text="\n".join(out) + "\n", n=n)


def pruned_network(mlp: MLP, dead_hidden: np.ndarray) -> MLP:
    """Delete the neurons flagged in a flat hidden-neuron mask (``prune_neurons``)."""
    from ..engine.prune import layer_slices

    sls = layer_slices(mlp.widths)
    return mlp.prune([np.asarray(dead_hidden[s], dtype=bool) for s in sls[:-1]])
