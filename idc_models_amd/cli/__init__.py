"""Command-line entry points with the reference scripts' positional arguments.

    python -m idc_models_amd.cli dist vgg   PATH          # dist_model_tf_vgg.py PATH
    python -m idc_models_amd.cli dist mobile PATH         # dist_model_tf_mobile.py PATH
    python -m idc_models_amd.cli dist dense PATH          # dist_model_tf_dense.py PATH
    python -m idc_models_amd.cli fed PATH ROUNDS iid|noniid      # fed_model.py
    python -m idc_models_amd.cli secure PATH ROUNDS PERCENT      # secure_fed_model.py

Multi-GPU data parallelism: launch with ``torchrun --nproc-per-node N --master-addr 127.0.0.1``
(one process per MI355X).  ``--config file.yaml`` loads one of ``configs/*.yaml``.
"""
from __future__ import annotations

import argparse
import json
import sys


def _load_config(path):
    if not path:
        return {}
    import yaml
    with open(path) as f:
        return yaml.safe_load(f) or {}


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(prog="idc_models_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    d = sub.add_parser("dist", help="two-phase data-parallel transfer learning")
    d.add_argument("preset", choices=["vgg", "mobile", "dense"])
    d.add_argument("path")
    d.add_argument("--config")
    d.add_argument("--strategy", default=None, choices=[None, "mirrored", "central", "one"])
    d.add_argument("--synthetic", action="store_true")
    d.add_argument("--epochs", type=int, default=None, help="initial (= fine-tune) epochs")
    d.add_argument("--steps-per-epoch", type=int, default=None)
    d.add_argument("--arch", default=None)
    f = sub.add_parser("fed", help="federated averaging (fed_model.py)")
    f.add_argument("path")
    f.add_argument("rounds", type=int)
    f.add_argument("iid")
    f.add_argument("--config")
    f.add_argument("--synthetic", action="store_true")
    f.add_argument("--arch", default=None)
    f.add_argument("--secure-agg", default=None, choices=[None, "mask"],
                   help="masked aggregation of the weighted deltas (secure FedAvg)")
    f.add_argument("--no-resume", action="store_true", help="ignore {path}/fed_state/state.pt")
    s = sub.add_parser("secure", help="secure federated learning (secure_fed_model.py)")
    s.add_argument("path")
    s.add_argument("rounds", type=int)
    s.add_argument("percent", type=float)
    s.add_argument("--config")
    s.add_argument("--mode", default=None, choices=[None, "mask", "paillier", "none"])
    s.add_argument("--synthetic", action="store_true")
    s.add_argument("--arch", default=None)
    s.add_argument("--clients", type=int, default=None)
    a = ap.parse_args(argv)
    cfg = _load_config(getattr(a, "config", None))

    if a.cmd == "dist":
        from ..recipes.transfer import PRESETS, TransferConfig, run_transfer_learning
        kw = dict(PRESETS[a.preset])
        kw.update(cfg)
        kw["path"] = a.path
        if a.strategy:
            kw["strategy"] = a.strategy
        if a.synthetic:
            kw["dataset"] = "synthetic"
        if a.epochs is not None:
            kw["initial_epochs"] = kw["fine_tune_epochs"] = a.epochs
        if a.steps_per_epoch is not None:
            kw["steps_per_epoch"] = a.steps_per_epoch
        if a.arch:
            kw["arch"] = a.arch
        if "input_shape" in kw:
            kw["input_shape"] = tuple(kw["input_shape"])
        run_transfer_learning(TransferConfig(**kw))
    elif a.cmd == "fed":
        from ..recipes.federated import FedConfig, run_fedavg
        kw = dict(cfg)
        kw.update(path=a.path, rounds=a.rounds, iid=(a.iid == "iid"))
        if a.synthetic:
            kw["synthetic"] = True
        if a.arch:
            kw["arch"] = a.arch
        if a.secure_agg:
            kw["secure_aggregation"] = a.secure_agg
        if a.no_resume:
            kw["resume"] = False
        if "input_shape" in kw:
            kw["input_shape"] = tuple(kw["input_shape"])
        run_fedavg(FedConfig(**kw))
    elif a.cmd == "secure":
        from ..recipes.federated import SecureConfig, run_secure
        kw = dict(cfg)
        kw.update(path=a.path, rounds=a.rounds, percent=a.percent)
        if a.mode:
            kw["mode"] = a.mode
        if a.synthetic:
            kw["synthetic"] = True
        if a.arch:
            kw["arch"] = a.arch
        if a.clients:
            kw["num_clients"] = a.clients
        if "input_shape" in kw:
            kw["input_shape"] = tuple(kw["input_shape"])
        run_secure(SecureConfig(**kw))
    return 0


if __name__ == "__main__":
    sys.exit(main())
