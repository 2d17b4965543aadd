"""Command line interface (replaces ``src/fairify.sh`` + the per-family copied driver scripts).

    python -m fairify_amd.cli presets
    python -m fairify_amd.cli verify --preset src/GC-age --models GC-1,GC-3 --out results/gc
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m fairify_amd.cli verify --preset stress/AC ...
    python -m fairify_amd.cli zoo [--import-dir /path/to/models]
    python -m fairify_amd.cli analyze --preset experiment/AC-3 --model AC-3 --fairer AC-3 ...
    python -m fairify_amd.cli repair --model AC-3 --counterexamples results/ac3/counterexamples.csv ...
    python -m fairify_amd.cli export-cex --preset src/AC-sex --model AC-3 --results results/ac

The reference's only flag is ``sys.argv[1]`` = soft timeout (src/AC/Verify-AC.py:147-148);
every other constant is a preset field here and can be overridden on the command line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from dataclasses import replace


def _device(arg):
    import torch

    if arg:
        return arg
    return "cuda" if torch.cuda.is_available() else "cpu"


def cmd_presets(args):
    from . import presets

    for name, p in sorted(presets.PRESETS.items()):
        g = p.grid()
        print(f"{name:20s} suite={p.suite:9s} PA={','.join(p.query.pa):22s} RA={','.join(p.query.ra) or '-':9s} "
              f"tau={p.query.tau:<2d} P={p.partition_size:<4d} partitions={len(g):<9d} soft={p.soft_timeout:g}s "
              f"hard={p.hard_timeout:g}s models={len(p.models)}  [{p.source}]")


def cmd_verify(args):
    import os

    from .parallel import balance as BL

    # several ranks per node (torchrun): each takes the CPUs local to its GPU (sysfs NUMA locality,
    # parallel/balance.py) for its host threads / HIP streams / LP workers, before the GPU is touched
    BL.pin_rank(int(os.environ.get("LOCAL_RANK", "0")),
                int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1"))))
    from . import presets
    from .engine.pipeline import VerifyConfig
    from .engine.runner import run_preset
    from .parallel import dist as D

    pre = presets.get(args.preset)
    if args.partition_size:
        pre = replace(pre, partition_size=args.partition_size)
    info = D.init(_device(args.device))
    cfg = VerifyConfig(sim_size=args.sim_size or pre.sim_size, seed=args.seed, chunk=args.chunk,
                       soft_timeout=args.soft_timeout if args.soft_timeout is not None else pre.soft_timeout,
                       hard_timeout=args.hard_timeout if args.hard_timeout is not None else pre.hard_timeout,
                       node_budget=args.node_budget, heuristic=not args.no_heuristic,
                       heuristic_p=args.heuristic_p if args.heuristic_p is not None else pre.heuristic_p,
                       heuristic_node_budget=args.node_budget, smt_backend=args.smt,
                       escalate_budget=args.escalate_budget, escalate_max_open=args.escalate_max_open,
                       escalate_probation=tuple(tuple(int(v) for v in st.split(":"))
                                                for st in args.escalate_probation.split(",") if st),
                       keep_masks=args.keep_masks, lp_budget=args.lp_budget, trust_milp=args.trust_milp)
    if args.residual_samples is not None:
        cfg.residual_samples = args.residual_samples
    models = args.models.split(",") if args.models else None
    run_preset(pre, models=models, weights=args.weights, out_dir=args.out, cfg=cfg, info=info,
               max_partitions=args.max_partitions, resume=args.resume, seed=args.seed,
               accuracy=not args.no_accuracy, escalate=args.escalate,
               concurrency=args.concurrency or (4 if info.device.type == "cuda" else 1),
               anytime_budget=(args.anytime_budget or cfg.hard_timeout) if args.anytime else None,
               metrics_csv=True if args.metrics_csv else None, balance=args.balance)
    D.destroy(info)


def cmd_zoo(args):
    from .models.zoo import ZOO, get_model, has_weights

    if args.import_dir:
        import subprocess

        tool = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "import_zoo.py")
        subprocess.run([sys.executable, tool, args.import_dir], check=True)
    for name, (suite, n_in, hidden) in sorted(ZOO.items()):
        print(f"{name:10s} suite={suite:9s} {n_in}->{'-'.join(map(str, hidden))}->1 "
              f"weights={'shipped' if has_weights(name) else 'random-only'}")


def cmd_analyze(args):
    from .analysis.report import analyze_model

    out = analyze_model(args.preset, args.model, fairer=args.fairer, results=args.results, weights=args.weights,
                        seed=args.seed, out_dir=args.out, device=_device(args.device),
                        causal_samples=args.causal_max)
    print(json.dumps(out, indent=2, default=float))


def cmd_repair(args):
    if args.method == "finetune":
        # GC/BM recipe: fine-tune on a synthetic CSV with early stopping (src/GC/new_model.py:8-58,
        # src/BM/new_model.py:8-40)
        from .models.zoo import get_model
        from .repair.finetune import finetune_csv

        if not args.data or not args.suite:
            raise SystemExit("--method finetune needs --data CSV and --suite german|bank")
        m = get_model(args.model, weights=args.weights, seed=args.seed)
        r = finetune_csv(m, args.data, args.suite, lr=args.lr, epochs=args.max_epochs, seed=args.seed,
                         device=_device(args.device), name=os.path.splitext(os.path.basename(args.out))[0])
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        r.model.save_npz(args.out if args.out.endswith(".npz") else args.out + ".npz")
        print(json.dumps({"model": args.model, "out": args.out, "epochs_run": r.epochs_run, "best_epoch": r.best_epoch,
                          "val_acc": r.val_acc, "val_loss": r.val_loss, "train_rows": r.train_rows,
                          "val_rows": r.val_rows}, indent=2))
        return
    from .repair.retrain import repair_model

    out = repair_model(args.model, counterexamples=args.counterexamples, method=args.method, out=args.out,
                       top_k=args.top_k, epochs=args.epochs, weights=args.weights, seed=args.seed,
                       device=_device(args.device))
    print(json.dumps(out, indent=2, default=float))


def cmd_export(args):
    from .report.counterexamples import export_counterexamples

    path = export_counterexamples(args.preset, args.model, args.results, out=args.out, weights=args.weights)
    print(path)


def cmd_export_smt(args):
    """Write the SMT-LIB2 query of partitions (sound-pruned on the box) for external solvers."""
    import numpy as np
    import torch

    from . import presets
    from .engine import prune as P_
    from .models.zoo import get_model
    from .ops.backend import Backend
    from .partition import processing_order
    from .smt import encode_partition, pruned_network

    pre = presets.get(args.preset)
    grid = pre.grid()
    q = pre.resolved()
    m = get_model(args.model, weights=args.weights, seed=args.seed)
    order = processing_order(grid, seed=args.seed)
    ids = order[:args.count] if args.ids is None else np.array([int(x) for x in args.ids.split(",")])
    lo, hi = grid.decode(ids)
    be = Backend(m, device=_device(args.device))
    r = be.bounds(torch.from_numpy(lo).float().to(be.device), torch.from_numpy(hi).float().to(be.device),
                  mode="ibp", keep_layers=True)
    nh = int(sum(m.hidden))
    dead = torch.cat(r.layer_ub, dim=1)[:, :nh] <= 0
    dead = P_.ensure_one_alive(torch.cat([dead, torch.zeros_like(dead[:, :1])], dim=1), m.widths)[:, :nh]
    dead = dead.cpu().numpy()
    os.makedirs(args.out, exist_ok=True)
    for k, gid in enumerate(ids):
        net = pruned_network(m, dead[k])
        text = encode_partition(net, q, lo[k], hi[k], timeout_s=args.timeout, fork_params=args.fork_params).text
        path = os.path.join(args.out, f"{args.model}-p{int(gid)}.smt2")
        with open(path, "w") as f:
            f.write(text)
        print(path, f"(pruned {m.n_neurons - net.n_neurons} of {m.n_neurons} neurons)")


def main(argv=None):
    ap = argparse.ArgumentParser(prog="fairify_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    sub.add_parser("presets").set_defaults(fn=cmd_presets)

    v = sub.add_parser("verify", help="verify a preset's models (torchrun for multi-GPU)")
    v.add_argument("--preset", required=True)
    v.add_argument("--models", default=None)
    v.add_argument("--weights", default="zoo", help="zoo | random | path/to/model.h5")
    v.add_argument("--out", default="results")
    v.add_argument("--partition-size", type=int, default=None)
    v.add_argument("--soft-timeout", type=float, default=None)
    v.add_argument("--hard-timeout", type=float, default=None)
    v.add_argument("--heuristic-p", type=float, default=None)
    v.add_argument("--no-heuristic", action="store_true")
    v.add_argument("--node-budget", type=int, default=4096)
    v.add_argument("--sim-size", type=int, default=None)
    v.add_argument("--chunk", type=int, default=4096)
    v.add_argument("--seed", type=int, default=0)
    v.add_argument("--max-partitions", type=int, default=None)
    v.add_argument("--resume", action="store_true")
    v.add_argument("--escalate", type=int, default=1,
                   help="retry each round's UNKNOWN partitions on all ranks with N x the node budget")
    v.add_argument("--escalate-budget", type=int, default=0,
                   help="second sound BaB pass with this node budget on each chunk's UNKNOWN residue")
    v.add_argument("--escalate-probation", default="",
                   help="inline escalation steps 'budget:max_open,...' between the node budget and "
                        "--escalate-budget (native BaB; bench default 2048:768,4096:768,8192:768,16384:1024 with --escalate-budget 32768)")
    v.add_argument("--escalate-max-open", type=int, default=0,
                   help="escalate only residue partitions that left <= this many open BaB nodes (0 = all)")
    v.add_argument("--balance", default="queue", choices=["queue", "strided"],
                   help="several ranks: claim units of each round from a shared atomic counter (queue, dynamic "
                        "load balance) or verify fixed strided shares (strided)")
    v.add_argument("--concurrency", type=int, default=0,
                   help="chunks verified at once per rank, one HIP stream each (default 4 on GPU, 1 on CPU)")
    v.add_argument("--smt", default="auto", help="host SMT back-end for the residue: auto | z3py | z3bin | none")
    v.add_argument("--lp-budget", type=int, default=4096,
                   help="without Z3 (--smt auto/milp): verified-LP branch-and-bound nodes per partition on the "
                        "residue, sound UNSAT (smt/lpbab.py); 0 = the HiGHS MILP, whose UNSAT is not a proof")
    v.add_argument("--trust-milp", action="store_true",
                   help="count HiGHS MILP UNSAT (floating-point dual bound) as verdicts (stage 'milp', excluded "
                        "from the sound figures); implies the MILP stage")
    v.add_argument("--anytime", action="store_true",
                   help="spend the per-model wall budget (--anytime-budget, default the preset's hard timeout) on "
                        "growing sound BaB budgets and falsifier rounds over the UNKNOWN residue")
    v.add_argument("--anytime-budget", type=float, default=None, help="seconds per model for --anytime")
    v.add_argument("--keep-masks", action="store_true",
                   help="gather every partition's final dead-neuron mask (packed bitset) to rank 0 and write "
                        "OUT/masks/<model>.npz with the unique masks (dedup) for pruned-subnet export")
    v.add_argument("--residual-samples", type=int, default=None)
    v.add_argument("--metrics-csv", action="store_true",
                   help="also write the per-partition metrics CSV of the experiment drivers "
                        "(on by default for experiment/* presets)")
    v.add_argument("--no-accuracy", action="store_true")
    v.add_argument("--device", default=None)
    v.set_defaults(fn=cmd_verify)

    z = sub.add_parser("zoo", help="list the model zoo / import Keras .h5 models")
    z.add_argument("--import-dir", default=None)
    z.set_defaults(fn=cmd_zoo)

    a = sub.add_parser("analyze", help="group metrics, causal discrimination, hybrid routing")
    a.add_argument("--preset", required=True)
    a.add_argument("--model", required=True)
    a.add_argument("--fairer", default=None)
    a.add_argument("--results", default=None, help="results dir of a verify run (partition verdicts)")
    a.add_argument("--weights", default="zoo")
    a.add_argument("--seed", type=int, default=0)
    a.add_argument("--out", default=None)
    a.add_argument("--causal-max", type=int, default=1000)
    a.add_argument("--device", default=None)
    a.set_defaults(fn=cmd_analyze)

    r = sub.add_parser("repair", help="bias localisation + masked fine-tune / counterexample retraining")
    r.add_argument("--model", required=True)
    r.add_argument("--counterexamples", default=None)
    r.add_argument("--method", default="masked", choices=["masked", "retrain", "finetune"])
    r.add_argument("--data", default=None, help="finetune: synthetic CSV (reference experimentData layout)")
    r.add_argument("--suite", default=None, choices=["german", "bank"], help="finetune: column spec")
    r.add_argument("--lr", type=float, default=5e-4)
    r.add_argument("--max-epochs", type=int, default=100, help="finetune: epochs before early stopping")
    r.add_argument("--out", required=True)
    r.add_argument("--top-k", type=int, default=10)
    r.add_argument("--epochs", type=int, default=5)
    r.add_argument("--weights", default="zoo")
    r.add_argument("--seed", type=int, default=0)
    r.add_argument("--device", default=None)
    r.set_defaults(fn=cmd_repair)

    e = sub.add_parser("export-cex", help="decode counterexamples of a verify run to category labels")
    e.add_argument("--preset", required=True)
    e.add_argument("--model", required=True)
    e.add_argument("--results", required=True)
    e.add_argument("--out", default=None)
    e.add_argument("--weights", default="zoo")
    e.set_defaults(fn=cmd_export)

    x = sub.add_parser("export-smt", help="write SMT-LIB2 partition queries (GPU-pruned) for external solvers")
    x.add_argument("--preset", required=True)
    x.add_argument("--model", required=True)
    x.add_argument("--out", required=True)
    x.add_argument("--count", type=int, default=4, help="first N partitions of the seeded order")
    x.add_argument("--ids", default=None, help="comma list of grid ids (overrides --count)")
    x.add_argument("--timeout", type=float, default=100.0)
    x.add_argument("--fork-params", action="store_true")
    x.add_argument("--weights", default="zoo")
    x.add_argument("--seed", type=int, default=0)
    x.add_argument("--device", default=None)
    x.set_defaults(fn=cmd_export_smt)

    args = ap.parse_args(argv)
    args.fn(args)


if __name__ == "__main__":
    main()
