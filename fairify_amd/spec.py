"""Query / domain specification for individual-fairness verification.

A *domain* is an ordered list of integer-valued features (the order is the network's input
order, i.e. the data-frame column order the reference feeds to Z3,
``src/AC/Verify-AC.py:131-132``).  A *query* adds the protected attributes (PA), the relaxed
attributes (RA) with their tolerance tau, and optional domain overrides ("targeted" runs).

Semantics (reference ``src/GC/Verify-GC.py:135-155`` and ``utils/verif_utils.py:781-798``):

* ``lo_i <= x_i <= hi_i`` for every feature i of the partition box;
* for every PA p: ``lo_p <= x'_p <= hi_p`` and ``x_p != x'_p`` (each PA must differ);
* for every RA r: ``|x_r - x'_r| <= tau`` (x'_r is *not* clipped to the box);
* every other attribute: ``x_a == x'_a``;
* violation: ``(N(x) < 0 and N(x') > 0) or (N(x) > 0 and N(x') < 0)`` on the pre-sigmoid logit.

Attributes listed in PA/RA that are not columns of the domain are ignored, exactly like the
reference (``relaxed/GC/Verify-GC.py:58`` lists ``marital-status`` which GC does not have).
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np


@dataclass(frozen=True)
class Feature:
    name: str
    lo: int
    hi: int

    @property
    def size(self) -> int:
        return self.hi - self.lo + 1


@dataclass(frozen=True)
class Domain:
    """Ordered integer feature domain of one dataset suite."""

    suite: str
    features: Tuple[Feature, ...]
    label: str = "label"

    @property
    def n(self) -> int:
        return len(self.features)

    @property
    def names(self) -> List[str]:
        return [f.name for f in self.features]

    def index(self, name: str) -> int:
        for i, f in enumerate(self.features):
            if f.name == name:
                return i
        raise KeyError(name)

    def has(self, name: str) -> bool:
        return any(f.name == name for f in self.features)

    def lo(self) -> np.ndarray:
        return np.array([f.lo for f in self.features], dtype=np.int64)

    def hi(self) -> np.ndarray:
        return np.array([f.hi for f in self.features], dtype=np.int64)

    def with_overrides(self, overrides: Dict[str, Tuple[int, int]]) -> "Domain":
        feats = []
        for f in self.features:
            if f.name in overrides:
                lo, hi = overrides[f.name]
                feats.append(Feature(f.name, int(lo), int(hi)))
            else:
                feats.append(f)
        return replace(self, features=tuple(feats))

    def range_dict(self) -> Dict[str, List[int]]:
        return {f.name: [f.lo, f.hi] for f in self.features}


@dataclass(frozen=True)
class Query:
    """Fairness query over a domain: protected attrs, relaxed attrs (+tau)."""

    pa: Tuple[str, ...]
    ra: Tuple[str, ...] = ()
    tau: int = 0

    def resolve(self, domain: Domain) -> "ResolvedQuery":
        pa_idx = [domain.index(a) for a in self.pa if domain.has(a)]
        ra_idx = [domain.index(a) for a in self.ra if domain.has(a) and a not in self.pa]
        if not pa_idx:
            raise ValueError(f"none of the protected attributes {self.pa} are in domain {domain.suite}")
        return ResolvedQuery(domain=domain, pa_idx=tuple(pa_idx), ra_idx=tuple(ra_idx), tau=int(self.tau))


@dataclass(frozen=True)
class ResolvedQuery:
    domain: Domain
    pa_idx: Tuple[int, ...]
    ra_idx: Tuple[int, ...]
    tau: int

    @property
    def n(self) -> int:
        return self.domain.n

    @property
    def relaxed(self) -> bool:
        return len(self.ra_idx) > 0 and self.tau > 0

    def free_mask(self) -> np.ndarray:
        """Features that are shared between x and x' (neither PA nor RA)."""
        m = np.ones(self.n, dtype=bool)
        m[list(self.pa_idx)] = False
        m[list(self.ra_idx)] = False
        return m

    def pa_values(self, lo: np.ndarray, hi: np.ndarray) -> np.ndarray:
        """All PA assignments inside a box: array [V, len(pa)] (product of PA ranges)."""
        rngs = [np.arange(int(lo[p]), int(hi[p]) + 1) for p in self.pa_idx]
        mesh = np.meshgrid(*rngs, indexing="ij")
        return np.stack([m.reshape(-1) for m in mesh], axis=1).astype(np.int64)

    def pa_pairs(self, values: np.ndarray) -> np.ndarray:
        """Ordered index pairs (v, v') whose PA components ALL differ: [P, 2]."""
        V = values.shape[0]
        diff = np.all(values[:, None, :] != values[None, :, :], axis=2)
        ii, jj = np.nonzero(diff)
        return np.stack([ii, jj], axis=1).astype(np.int64) if V else np.zeros((0, 2), np.int64)


# --------------------------------------------------------------------------------------
# Suite domains (feature order = network input order; ranges = the reference `src/` presets)
# --------------------------------------------------------------------------------------

def _dom(suite: str, label: str, items: Sequence[Tuple[str, int, int]]) -> Domain:
    return Domain(suite=suite, features=tuple(Feature(n, int(lo), int(hi)) for n, lo, hi in items), label=label)


# Adult census: src/AC/Verify-AC.py:44-58 ; column order utils/verif_utils.py:119-190
ADULT = _dom("adult", "income-per-year", [
    ("age", 10, 100), ("workclass", 0, 6), ("education", 0, 15), ("education-num", 1, 16),
    ("marital-status", 0, 6), ("occupation", 0, 13), ("relationship", 0, 5), ("race", 0, 4),
    ("sex", 0, 1), ("capital-gain", 0, 19), ("capital-loss", 0, 19), ("hours-per-week", 1, 100),
    ("native-country", 0, 40),
])

# German credit: src/GC/Verify-GC.py:40-60 ; sex appended last (utils/standard_data.py:4-65)
GERMAN = _dom("german", "credit", [
    ("status", 0, 2), ("month", 0, 80), ("credit_history", 0, 2), ("purpose", 0, 9),
    ("credit_amount", 0, 20000), ("savings", 0, 2), ("employment", 0, 2),
    ("investment_as_income_percentage", 1, 4), ("other_debtors", 0, 2), ("residence_since", 1, 4),
    ("property", 0, 2), ("age", 0, 1), ("installment_plans", 0, 2), ("housing", 0, 2),
    ("number_of_credits", 1, 4), ("skill_level", 0, 3), ("people_liable_for", 1, 2),
    ("telephone", 0, 1), ("foreign_worker", 0, 1), ("sex", 0, 1),
])

# Bank marketing: src/BM/Verify-BM.py:33-48 ; column order utils/verif_utils.py:309-366
BANK = _dom("bank", "y", [
    ("age", 0, 1), ("job", 0, 10), ("marital", 0, 2), ("education", 0, 6), ("default", 0, 1),
    ("housing", 0, 1), ("loan", 0, 1), ("contact", 0, 1), ("month", 0, 11), ("day_of_week", 0, 6),
    ("duration", 0, 5000), ("emp.var.rate", -3, 1), ("campaign", 1, 50), ("pdays", 0, 999),
    ("previous", 0, 7), ("poutcome", 0, 2),
])

# COMPAS 6-feature variant: src/CP/Verify-CP.py:49-54
COMPAS = _dom("compas", "score_factor", [
    ("Two_yr_Recidivism", 0, 1), ("Number_of_Priors", 0, 38), ("Age", 0, 1), ("Race", 0, 1),
    ("Female", 0, 1), ("Misdemeanor", 0, 1),
])

# COMPAS 12-feature variant used by CP-2..10 / aCP-1-Old (commented block src/CP/Verify-CP.py:57-68)
COMPAS12 = _dom("compas12", "label", [
    ("sex", 0, 1), ("age", 0, 2), ("race", 0, 1), ("d", 0, 10), ("e", 0, 9), ("f", 0, 36),
    ("g", 0, 1), ("h", 0, 1), ("i", 0, 1), ("j", 0, 9), ("k", 0, 9), ("l", 0, 36),
])

# Default credit: src/DF/Verify-DF.py:54-83 (float ranges, Int Z3 variables -> integer lattice)
DEFAULT = _dom("default", "default.payment.next.month", [
    ("LIMIT_BAL", 10000, 1000000), ("AGE", 21, 79),
    ("PAY_1", 0, 1), ("PAY_2", 0, 1), ("PAY_3", 0, 1), ("PAY_4", 0, 1), ("PAY_5", 0, 1), ("PAY_6", 0, 1),
    ("BILL_AMT1", -165580, 964511), ("BILL_AMT2", -69777, 983931), ("BILL_AMT3", -157264, 1664089),
    ("BILL_AMT4", -170000, 891586), ("BILL_AMT5", -81334, 927171), ("BILL_AMT6", -339603, 961664),
    ("PAY_AMT1", 0, 873552), ("PAY_AMT2", 0, 1684259), ("PAY_AMT3", 0, 896040),
    ("PAY_AMT4", 0, 621000), ("PAY_AMT5", 0, 426529), ("PAY_AMT6", 0, 528666),
    ("SEX_2", 0, 1), ("EDUCATION_1", 0, 1), ("EDUCATION_2", 0, 1), ("EDUCATION_3", 0, 1),
    ("EDUCATION_4", 0, 1), ("EDUCATION_5", 0, 1), ("EDUCATION_6", 0, 1),
    ("MARRIAGE_1", 0, 1), ("MARRIAGE_2", 0, 1), ("MARRIAGE_3", 0, 1),
])

DOMAINS: Dict[str, Domain] = {d.suite: d for d in (ADULT, GERMAN, BANK, COMPAS, COMPAS12, DEFAULT)}

# Grid attribute order used by the reference partitioner (dict order of the driver's
# range_dict); only affects partition numbering, kept for id-level parity.
BANK_GRID_ORDER = ("job", "marital", "education", "default", "housing", "loan", "contact", "month",
                   "day_of_week", "emp.var.rate", "duration", "campaign", "pdays", "previous",
                   "poutcome", "age")


def domain(suite: str) -> Domain:
    return DOMAINS[suite]
