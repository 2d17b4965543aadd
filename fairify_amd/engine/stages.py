"""Which pipeline stage decided a partition, and which of those verdicts are sound.

One registry for the wire format (``parallel/wire.py``), the packed CSV rows and Table-V rows
(``engine/runner.py``) and the bench JSON (``bench.py``); the code of a stage is its index here
(append only: checkpoints and wire buffers store the index).

Verdict / stage combinations:

* ``sim``, ``falsify``, ``bab``, ``relu``, ``smt``, ``heuristic-confirmed`` SAT: a concrete pair
  confirmed exactly on the ORIGINAL network (pair constraints + rigorous fp64 / rational logits).
* ``bab`` UNSAT: every node of the partition closed by a rigorous input-split certificate.
* ``relu`` UNSAT: closed by the ReLU phase-split search (engine/relu_bab.py), rigorous bounds.
* ``beta`` UNSAT: closed by the beta-CROWN phase-split search (engine/beta_bab.py): every node's
  Lagrangian bound re-evaluated in fp64 with rigorous rounding terms; SAT: a confirmed pair.
* ``smt`` UNSAT: Z3 (exact rational arithmetic), when installed.
* ``lp`` UNSAT: verified-LP branch-and-bound (smt/lpbab.py): HiGHS LP relaxations, every closed
  node certified by a rigorously evaluated weak-duality bound from the solver's multipliers;
  ``lp`` SAT: a lattice point confirmed exactly.
* ``milp``: HiGHS MILP on the residue.  Its UNSAT rests on a floating-point dual bound, so by
  default it is NOT a verdict: the partition stays UNKNOWN with stage ``milp`` (the solver's
  claim is recorded, unverified); ``VerifyConfig.trust_milp`` restores the round-2 behaviour
  (UNSAT with stage ``milp``, excluded from every sound count).
* ``heuristic`` SAT / UNSAT: the reference's unsound heuristic-pruning retry
  (src/AC/Verify-AC.py:173-212): UNSAT holds for the pruned net only, SAT flips the pruned net
  but not the original (a SAT that flips the original is promoted to ``heuristic-confirmed``).
"""
from __future__ import annotations

STAGES = ("", "sim", "bab", "heuristic", "smt", "falsify", "milp", "heuristic-confirmed", "relu", "lp", "beta")
CODE = {s: k for k, s in enumerate(STAGES)}

SOUND_SAT = frozenset({"sim", "bab", "falsify", "smt", "milp", "heuristic-confirmed", "relu", "lp", "beta", ""})
SOUND_UNSAT = frozenset({"bab", "smt", "relu", "lp", "beta", ""})
UNSOUND_UNSAT = frozenset({"heuristic", "milp"})


def code(stage: str) -> int:
    return CODE.get(stage, 0)


def is_sound(verdict: str, stage: str) -> bool:
    """Whether a decided (sat / unsat) verdict is sound for the original network."""
    if verdict == "sat":
        return stage != "heuristic"
    if verdict == "unsat":
        return stage not in UNSOUND_UNSAT
    return False
