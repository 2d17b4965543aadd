"""Experiment presets: every driver configuration of the reference.

The reference encodes each experiment family as a copied script differing only in module-level
constants (e.g. ``src/AC/Verify-AC.py:34-71``, ``stress/AC/Verify-AC.py:21-56``,
``relaxed/BM/Verify-BM.py:21-54``, ``targeted2/GC/Verify-GC.py:21-58``).  Here each is one
declarative ``Preset``; ``fairify_amd.cli verify --preset <name>`` reproduces the run.
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Dict, List, Optional, Tuple

from .models.zoo import SUITE_MODELS
from .partition import Grid
from .spec import BANK_GRID_ORDER, DOMAINS, Domain, Query


@dataclass(frozen=True)
class Preset:
    name: str
    suite: str                                  # domain key
    query: Query
    partition_size: int
    soft_timeout: float = 100.0
    hard_timeout: float = 30 * 60.0
    heuristic_p: float = 5.0
    sim_size: int = 1000
    models: Tuple[str, ...] = ()
    overrides: Tuple[Tuple[str, int, int], ...] = ()
    capped: Optional[int] = None                # partitioned_ranges_df max_partitions
    grid_order: Optional[Tuple[str, ...]] = None
    source: str = ""

    def domain(self) -> Domain:
        d = DOMAINS[self.suite]
        if self.overrides:
            d = d.with_overrides({n: (lo, hi) for n, lo, hi in self.overrides})
        return d

    def grid(self, seed: int = 0) -> Grid:
        d = self.domain()
        if self.capped:
            return Grid.capped(d, self.partition_size, list(self.query.pa), self.capped, seed=seed)
        order = None
        if self.grid_order:
            order = [a for a in self.grid_order if d.has(a)]
        return Grid.reference(d, self.partition_size, order=order)

    def resolved(self):
        return self.query.resolve(self.domain())


AC = tuple(SUITE_MODELS["AC"])
BM = tuple(SUITE_MODELS["BM"])
GC = tuple(SUITE_MODELS["GC"])

PRESETS: Dict[str, Preset] = {}


def _add(p: Preset):
    PRESETS[p.name] = p


# ---- src/ (paper Table V) -------------------------------------------------------------------
_add(Preset("src/AC-sex", "adult", Query(("sex",)), 10, 100, 1800, 5, 1000, AC, source="src/AC/Verify-AC.py:34-71"))
_add(Preset("src/AC-race", "adult", Query(("race",)), 10, 100, 1800, 5, 1000, AC, source="src/AC/Verify-AC.py:34-71"))
_add(Preset("src/GC-age", "german", Query(("age",)), 100, 100, 1800, 5, 1000, GC, source="src/GC/Verify-GC.py:29-71"))
_add(Preset("src/GC-sex", "german", Query(("sex",)), 100, 100, 1800, 5, 1000, GC, source="src/GC/Verify-GC.py:29-71"))
_add(Preset("src/BM-age", "bank", Query(("age",)), 100, 100, 1800, 5, 1000, BM, grid_order=BANK_GRID_ORDER,
            source="src/BM/Verify-BM.py:21-46"))
_add(Preset("src/CP", "compas", Query(("Race",)), 5, 100, 1800, 50, 10000, ("CP-1", "CP-11"),
            source="src/CP/Verify-CP.py:36-79"))
_add(Preset("src/CP12", "compas12", Query(("race",)), 5, 100, 1800, 50, 10000,
            tuple(f"CP-{k}" for k in range(2, 11)) + ("aCP-1-Old",), source="src/CP/Verify-CP.py:57-68"))
_add(Preset("src/DF", "default", Query(("SEX_2",)), 8, 100, 3600, 100, 1000, tuple(SUITE_MODELS["DF"]), capped=100,
            source="src/DF/Verify-DF.py:41-98"))
# ---- stress/ ----------------------------------------------------------------------------------
_add(Preset("stress/AC", "adult", Query(("sex",)), 6, 200, 3600, 20, 1000, AC, source="stress/AC/Verify-AC.py:21-56"))
_add(Preset("stress/GC", "german", Query(("age",)), 10, 200, 3600, 20, 1000, GC, source="stress/GC/Verify-GC.py:29-71"))
_add(Preset("stress/BM", "bank", Query(("age",)), 10, 200, 3600, 20, 1000, BM, grid_order=BANK_GRID_ORDER,
            source="stress/BM/Verify-BM.py:21-46"))
# ---- relaxed/ ---------------------------------------------------------------------------------
_add(Preset("relaxed/AC", "adult", Query(("race",), ("age",), 5), 6, 100, 3600, 20, 1000, AC,
            source="relaxed/AC/Verify-AC.py:21-51"))
_add(Preset("relaxed/GC", "german", Query(("sex", "marital-status")), 10, 100, 3600, 20, 1000, GC,
            source="relaxed/GC/Verify-GC.py:25-60"))
_add(Preset("relaxed/BM", "bank", Query(("age",), ("duration",), 5), 10, 100, 3600, 20, 1000, BM,
            grid_order=BANK_GRID_ORDER, source="relaxed/BM/Verify-BM.py:21-54"))
# ---- targeted/ --------------------------------------------------------------------------------
_add(Preset("targeted/AC", "adult", Query(("race",)), 6, 100, 3600, 20, 1000, AC, overrides=(("age", 30, 35),),
            source="targeted/AC/Verify-AC.py:22-51"))
_add(Preset("targeted/GC", "german", Query(("sex",)), 10, 100, 3600, 20, 1000, GC,
            overrides=(("number_of_credits", 2, 2),), source="targeted/GC/Verify-GC.py:30-66"))
_add(Preset("targeted/BM", "bank", Query(("age",), ("duration",), 5), 10, 100, 3600, 20, 1000, BM,
            overrides=(("job", 2, 2), ("loan", 1, 1)), grid_order=BANK_GRID_ORDER,
            source="targeted/BM/Verify-BM.py:22-54"))
# ---- targeted2/ -------------------------------------------------------------------------------
_add(Preset("targeted2/AC", "adult", Query(("race",)), 6, 100, 3600, 20, 1000, AC,
            overrides=(("education", 9, 10),), source="targeted2/AC/Verify-AC.py:22-51"))
_add(Preset("targeted2/GC", "german", Query(("sex", "marital-status")), 10, 100, 3600, 20, 1000, GC,
            overrides=(("purpose", 7, 7), ("foreign_worker", 0, 0)), source="targeted2/GC/Verify-GC.py:21-58"))
_add(Preset("targeted2/BM", "bank", Query(("age",), ("duration",), 5), 10, 100, 3600, 20, 1000, BM,
            overrides=(("poutcome", 2, 2),), grid_order=BANK_GRID_ORDER, source="targeted2/BM/Verify-BM.py:22-54"))
# ---- fork experiment drivers ------------------------------------------------------------------
_add(Preset("experiment/AC-3", "adult", Query(("sex",)), 30, 100, 1800, 100, 1000, ("AC-3",),
            source="src/AC/Verify-AC-experiment-new2.py:42-78"))
_add(Preset("experiment/GC-1", "german", Query(("age",)), 100, 100, 60, 5, 1000, ("GC-1",),
            source="src/GC/Verify-GC-experiment-new2.py:43-49"))
_add(Preset("experiment/BM", "bank", Query(("age",)), 10, 300, 3600, 100, 1000, ("BM-10",),
            source="src/BM/Verify-BM-experiment.py:35-41"))


def get(name: str) -> Preset:
    if name not in PRESETS:
        raise KeyError(f"unknown preset {name}; known: {', '.join(sorted(PRESETS))}")
    return PRESETS[name]
