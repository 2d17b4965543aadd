"""Host-side SMT subsystem: SMT-LIB2 encoding of the partition query, solver back-ends,
model parsing and an exact evaluator (test oracle).  See :mod:`fairify_amd.smt.encode`."""
from .encode import encode_partition, pruned_network, rational  # noqa: F401
from .sexpr import Evaluator, model_to_pair, parse_model  # noqa: F401
from .solver import available, resolve, solve  # noqa: F401
