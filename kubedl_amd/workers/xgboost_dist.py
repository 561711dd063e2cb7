"""XGBoostJob worker: distributed histogram GBDT on MI355X (one GPU per rank).

Accepts the reference example's arguments
(``example/xgboost/xgboostjob_v1alpha1_iris_train.yaml``):
``--job_type=Train --xgboost_parameter=objective:multi:softprob,num_class:3
--n_estimators=10 --learning_rate=0.1 --model_path=... --model_storage_type=oss``.

Rendezvous uses the env the XGBoost controller injects (``MASTER_ADDR``,
``MASTER_PORT``, ``WORLD_SIZE``); because the reference gives master-0 and
worker-0 the same ``RANK`` (a rabit-ism, ``controllers/xgboost/pod.go:112-143``)
the process-group rank comes from ``KDL_RANK`` when present.

Data: ``--dataset iris`` (scikit-learn's bundled copy; every rank takes a
row shard) or ``--dataset synthetic`` (``--rows`` x ``--features`` float
rows per rank with a nonlinear target, HIGGS-like shape).  Prints one JSON
line with the training metric and rounds/s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

from kubedl_amd.models.gbdt import GBDTParams, HistGBDT
from kubedl_amd.parallel import dist as kdist
from kubedl_amd.workers import common


def load_data(args, rank: int, world: int):
    if args.dataset == "iris":
        try:
            from sklearn.datasets import load_iris
            X, y = load_iris(return_X_y=True)
            X = torch.tensor(X, dtype=torch.float32)
            y = torch.tensor(y)
        except Exception:  # no sklearn: iris-shaped synthetic
            g = torch.Generator().manual_seed(0)
            y = torch.arange(150) % 3
            X = torch.randn(150, 4, generator=g) + y[:, None].float()
        return X[rank::world].contiguous(), y[rank::world].contiguous()
    g = torch.Generator().manual_seed(1234 + rank)
    X = torch.randn(args.rows, args.features, generator=g)
    logit = X[:, 0] * 1.5 - X[:, 1] ** 2 + X[:, 2] * X[:, 3] + 0.5 * torch.sin(3 * X[:, 4 % args.features])
    if args.objective_hint == "binary":
        y = (logit + 0.3 * torch.randn(args.rows, generator=g) > 0).long()
    else:
        y = logit + 0.1 * torch.randn(args.rows, generator=g)
    return X, y


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--job_type", default="Train")
    ap.add_argument("--xgboost_parameter", default="")
    ap.add_argument("--n_estimators", type=int, default=10)
    ap.add_argument("--learning_rate", type=float, default=0.3)
    ap.add_argument("--max_depth", type=int, default=6)
    ap.add_argument("--max_bin", type=int, default=256)
    ap.add_argument("--model_path", default="")
    ap.add_argument("--model_storage_type", default="local")
    ap.add_argument("--oss_param", default="")
    ap.add_argument("--dataset", default=None, choices=[None, "iris", "synthetic"])
    ap.add_argument("--rows", type=int, default=200000)
    ap.add_argument("--features", type=int, default=28)
    ap.add_argument("--objective_hint", default="binary", choices=["binary", "reg"])
    ap.add_argument("--cpu", action="store_true")
    args, _unknown = ap.parse_known_args(argv)
    if os.environ.get("KDL_RANK"):
        os.environ["RANK"] = os.environ["KDL_RANK"]
    info = kdist.init_from_env("cpu" if args.cpu else None)
    common.signal_ready({"rank": info.rank})
    if args.dataset is None:
        args.dataset = "iris" if "num_class:3" in args.xgboost_parameter else "synthetic"
    default_obj = "binary:logistic" if args.objective_hint == "binary" else "reg:squarederror"
    params = GBDTParams.parse(args.xgboost_parameter or f"objective:{default_obj}",
                              n_estimators=args.n_estimators, learning_rate=args.learning_rate,
                              max_depth=args.max_depth, max_bin=args.max_bin)
    if args.dataset == "iris" and params.max_bin > 64:
        params.max_bin = 64
    X, y = load_data(args, info.rank, info.world_size)
    model = HistGBDT(params, info.device)
    t0 = time.perf_counter()
    pred = model.fit(X, y, callback=lambda it, _p: common.report_progress(
        it + 1, final=it + 1 == params.n_estimators))
    if info.device.type == "cuda":
        torch.cuda.synchronize()
    dt = kdist.all_reduce_max(time.perf_counter() - t0, info)
    met = model.metric(pred, y.to(info.device))
    out = {"rank": info.rank, "world_size": info.world_size, "objective": params.objective,
           "rounds": params.n_estimators, "rows_per_rank": int(X.shape[0]), "features": int(X.shape[1]),
           "seconds": dt, "fit_rounds_per_sec": params.n_estimators / dt if dt > 0 else 0.0,
           # boosting rounds alone (setup = H2D copy + cuts + quantisation, reported apart)
           "rounds_per_sec": (params.n_estimators / model.stats["boost_s"]
                              if model.stats.get("boost_s", 0) > 0 else 0.0),
           "device": str(info.device), "hip_kernels": model.use_hip, **met, **model.stats}
    if info.rank == 0:
        print(json.dumps(out), flush=True)
        if args.model_path:
            path = args.model_path
            if args.model_storage_type != "local" or not os.path.isabs(path):
                # no object store on the node: keep the model in the pod sandbox
                path = os.path.join(os.environ.get("KDL_SANDBOX", "."), "model", path.strip("/"))
            os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
            with open(path + ".json", "w") as f:
                json.dump({"params": params.__dict__, "cuts": model.cuts.cpu().tolist(),
                           "trees": [[t.__dict__ for t in r] for r in model.trees]}, f)
    kdist.shutdown(info)
    return 0


if __name__ == "__main__":
    from kubedl_amd.parallel.dist import run_rank
    sys.exit(run_rank(main))
