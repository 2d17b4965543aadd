"""Host SMT back-ends for the residual partitions (optional; the GPU BaB is the default).

The reference's only decision procedure is Z3 (src/AC/Verify-AC.py:145-158).  Here the
solver is a pluggable host back-end that receives the SMT-LIB2 script of a GPU-pruned
subnetwork (:mod:`fairify_amd.smt.encode`):

* ``z3py``  — the ``z3`` Python module, if importable (``z3.Solver().from_string``);
* ``z3bin`` — a ``z3`` (or ``$FAIRIFY_SMT_BIN``) executable on PATH, fed the script on stdin;
* ``milp``  — HiGHS mixed-integer programming through SciPy, fed the GPU's rigorous layer
  bounds (:mod:`fairify_amd.smt.milp`; not an SMT-LIB consumer, the pipeline calls it directly);
* ``none``  — no solver: residual partitions stay UNKNOWN.

Neither Z3 flavour exists in this image; :func:`available` reports what was found and the
pipeline silently keeps ``none``.  Results come back as ``("sat", (x, x'))``,
``("unsat", None)`` or ``("unknown", None)`` — every ``sat`` is still re-confirmed with the
exact checker before it is reported (``C-check`` / ``V-accurate`` semantics).
"""
from __future__ import annotations

import os
import shutil
import subprocess
from typing import List, Optional, Tuple

from .sexpr import model_to_pair, parse_model

Result = Tuple[str, Optional[Tuple[List[int], List[int]]]]


def _z3py():
    try:
        import z3  # noqa: F401

        return z3
    except Exception:
        return None


def _z3bin() -> Optional[str]:
    return os.environ.get("FAIRIFY_SMT_BIN") or shutil.which("z3")


def available() -> List[str]:
    """Installed back-ends in preference order (Z3 first: exact arithmetic; then the HiGHS MILP
    back-end of :mod:`fairify_amd.smt.milp`, which SciPy ships)."""
    out = []
    if _z3py() is not None:
        out.append("z3py")
    if _z3bin():
        out.append("z3bin")
    from . import milp

    if milp.available():
        out.append("milp")
    return out


def resolve(backend: str = "auto") -> str:
    if backend == "none":
        return "none"
    have = available()
    if backend == "auto":
        return have[0] if have else "none"
    if backend not in have:
        raise RuntimeError(f"SMT back-end {backend!r} not available (found: {have or 'none'})")
    return backend


def solve(script: str, n: int, backend: str, timeout_s: float) -> Result:
    """Run one encoded partition query."""
    if backend == "none":
        return "unknown", None
    if backend == "z3py":
        z3 = _z3py()
        s = z3.Solver()
        s.set("timeout", int(timeout_s * 1000))
        body = "\n".join(l for l in script.splitlines() if not l.startswith(("(check-sat", "(get-model")))
        s.from_string(body)
        r = s.check()
        if r == z3.sat:
            m = s.model()
            model = {}
            for d in m.decls():
                v = m[d]
                if z3.is_int_value(v):
                    model[d.name()] = v.as_long()
            return "sat", model_to_pair(model, n)
        return ("unsat", None) if r == z3.unsat else ("unknown", None)
    if backend == "z3bin":
        exe = _z3bin()
        try:
            p = subprocess.run([exe, "-in", "-smt2", f"-T:{max(1, int(timeout_s + 1))}"], input=script,
                               capture_output=True, text=True, timeout=timeout_s + 5)
        except subprocess.TimeoutExpired:
            return "unknown", None
        out = p.stdout.strip()
        first = out.split("\n", 1)[0].strip() if out else ""
        if first == "sat":
            return "sat", model_to_pair(parse_model(out.split("\n", 1)[1] if "\n" in out else ""), n)
        if first == "unsat":
            return "unsat", None
        return "unknown", None
    raise ValueError(backend)
