"""End-to-end recipe smoke tests through the CLI on synthetic data (CPU, tiny sizes)."""
import os

import pytest
import yaml

from idc_models_amd.cli import main


def _cfg(tmp_path, name, d):
    p = tmp_path / name
    p.write_text(yaml.safe_dump(d))
    return str(p)


def test_dist_transfer_two_phase(tmp_path, capsys):
    cfg = _cfg(tmp_path, "t.yaml", dict(synthetic_size=160, batch_size=16, validation_steps=1,
                                        input_shape=[32, 32, 3], strategy="one"))
    assert main(["dist", "mobile", str(tmp_path), "--synthetic", "--epochs", "1",
                 "--steps-per-epoch", "1", "--config", cfg]) == 0
    out = capsys.readouterr().out
    assert "Pre-training with 1 devices took" in out
    assert "Fine-tuning with 1 devices took" in out
    assert "Number of layers in the base model:  155" in out
    assert os.path.exists(tmp_path / "logs" / "plot_dev1.png")


def test_fed_pretrain_checkpoint_then_rounds(tmp_path, capsys):
    cfg = _cfg(tmp_path, "f.yaml", dict(dataset_size=200, batch_size=20, pretrain_epochs=1,
                                        input_shape=[32, 32, 3], arch="mobilenetv2"))
    assert main(["fed", str(tmp_path), "1", "noniid", "--synthetic", "--config", cfg]) == 0
    out = capsys.readouterr().out
    assert os.path.exists(tmp_path / "pretrained" / "cp.h5")
    assert "Initial model:" in out and " 0, " in out
    # second run loads the checkpoint instead of pre-training (fixes quirk Q7)
    main(["fed", str(tmp_path), "1", "iid", "--synthetic", "--config", cfg])
    assert "Loading pretrained model" in capsys.readouterr().out


def test_fed_resume_and_secure_aggregation(tmp_path, capsys):
    """Federated resume (server state + round counter + RNG saved every round) and the masked
    weighted-delta aggregation through the CLI: a 1-round run, then a 2-round run continues at
    round 1 instead of starting over."""
    cfg = _cfg(tmp_path, "f.yaml", dict(dataset_size=200, batch_size=20, pretrain_epochs=1,
                                        input_shape=[32, 32, 3], arch="mobilenetv2"))
    assert main(["fed", str(tmp_path), "1", "iid", "--synthetic", "--secure-agg", "mask", "--config", cfg]) == 0
    out = capsys.readouterr().out
    assert " 0, " in out and os.path.exists(tmp_path / "fed_state" / "state.pt")
    assert main(["fed", str(tmp_path), "2", "iid", "--synthetic", "--secure-agg", "mask", "--config", cfg]) == 0
    out = capsys.readouterr().out
    assert "Resuming federated training at round 1" in out
    assert " 1, " in out and " 0, " not in out
    from idc_models_amd.fed import load_server_state
    assert load_server_state(str(tmp_path / "fed_state" / "state.pt")).round_num == 2


@pytest.mark.parametrize("mode", ["mask", "none"])
def test_secure_round(tmp_path, capsys, mode):
    cfg = _cfg(tmp_path, "s.yaml", dict(dataset_size=200, epochs=1))
    assert main(["secure", str(tmp_path), "2", "0.5", "--synthetic", "--mode", mode, "--config", cfg]) == 0
    out = capsys.readouterr().out.strip().splitlines()
    assert any("Secure fed model took" in l for l in out)
    assert len([l for l in out if len(l.split()) == 3]) >= 2  # "loss acc auc" per round


@pytest.mark.parametrize("name,kind", [("mobilenetv2_cpu", "dist"), ("vgg16_dp8", "dist"),
                                       ("densenet121_dp8", "dist"), ("fedavg_mobilenetv2_8", "fed"),
                                       ("secure_densenet121_8", "secure")])
def test_north_star_configs_are_valid(name, kind):
    """Every configs/*.yaml key is a field of its recipe's config dataclass."""
    import dataclasses
    import os
    from idc_models_amd.recipes import FedConfig, SecureConfig, TransferConfig
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "configs", name + ".yaml")) as f:
        cfg = yaml.safe_load(f)
    cls = {"dist": TransferConfig, "fed": FedConfig, "secure": SecureConfig}[kind]
    fields = {f.name for f in dataclasses.fields(cls)}
    assert set(cfg) <= fields, set(cfg) - fields
    if "input_shape" in cfg:
        cfg["input_shape"] = tuple(cfg["input_shape"])
    cls(**cfg)


def test_mobilenetv2_cpu_config_runs(tmp_path, capsys):
    """North-star config 1 end to end on the CPU (shortened: 1 step per phase, synthetic data)."""
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    assert main(["dist", "mobile", str(tmp_path), "--synthetic", "--epochs", "1", "--steps-per-epoch", "1",
                 "--config", os.path.join(root, "configs", "mobilenetv2_cpu.yaml")]) == 0
    assert "Fine-tuning with 1 devices took" in capsys.readouterr().out
