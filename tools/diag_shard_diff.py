"""Which partitions change verdict when a model's partitions are verified in different chunk
compositions (whole list vs strided halves)?  Prints the differing partitions' stages."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from fairify_amd import presets  # noqa: E402
from fairify_amd.engine.pipeline import VerifyConfig, verify_chunk  # noqa: E402
from fairify_amd.models.zoo import get_model  # noqa: E402
from fairify_amd.ops.backend import Backend  # noqa: E402
from fairify_amd.partition import processing_order  # noqa: E402

models = sys.argv[1].split(",") if len(sys.argv) > 1 else ["AC-8", "AC-3"]
limit = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
pre = presets.get("src/AC-sex")
grid, q = pre.grid(), pre.resolved()
order = processing_order(grid, 0)[:limit]
dev = torch.device("cuda")
cfg = VerifyConfig(sim_size=1000, chunk=4096, node_budget=512, heuristic=True, heuristic_node_budget=512,
                   escalate_budget=8192, escalate_max_open=384)
for name in models:
    m = get_model(name, weights="random", seed=0)
    be = Backend(m, dev)
    full = verify_chunk(be, m, q, grid, order, cfg)
    halves = [verify_chunk(be, m, q, grid, order[r::2], cfg) for r in range(2)]
    v = np.empty(len(order), dtype=object)
    st = np.empty(len(order), dtype=object)
    for r in range(2):
        v[r::2] = halves[r].cols["verdict"]
        st[r::2] = halves[r].cols["stage"]
    diff = np.nonzero(v != full.cols["verdict"])[0]
    from fairify_amd.engine.bab import STATS
    print(name, "differ:", len(diff), "bab stats", STATS, flush=True)
    for i in diff[:20]:
        print("  pos", i, "grid", order[i], "full", full.cols["verdict"][i], full.cols["stage"][i],
              "nodes", full.cols["nodes"][i], "| halves", v[i], st[i], flush=True)
