"""bench.py's launcher contract: ``--gpus N`` with no launcher environment
starts N rank processes itself and the job reports ``world_size == N``; a rank whose world is not N
refuses to run.  CPU ranks over gloo here; on GPUs the same ranks use RCCL."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=300)


def test_bench_spawns_requested_world_on_cpu():
    r = _run(["--gpus", "2", "--device", "cpu", "--model", "mobilenetv2", "--batch", "4", "--steps", "1",
              "--warmup", "0", "--fit-steps", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints exactly one line
    out = lines[0]
    assert out["config"]["world_size"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["comm_backend"] == "gloo"
    assert out["config"]["global_batch"] == 8 and out["steps"] == 1


def test_bench_spawns_world4_on_cpu():
    """The driver's N=4 point, rehearsed on gloo: 4 ranks, one JSON line, dp4, global batch 4x."""
    r = _run(["--gpus", "4", "--device", "cpu", "--model", "mobilenetv2", "--batch", "2", "--steps", "1",
              "--warmup", "0", "--fit-steps", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = lines[0]
    assert out["config"]["world_size"] == 4 and out["config"]["parallelism"] == "dp4"
    assert out["config"]["global_batch"] == 8


def test_bench_refuses_mismatched_world():
    r = _run(["--gpus", "4", "--device", "cpu", "--model", "mobilenetv2", "--batch", "4", "--steps", "1",
              "--warmup", "0", "--fit-steps", "0"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 3
    assert "error" in json.loads(r.stdout.strip().splitlines()[-1])


def test_bench_densenet201_cifar_phases_on_cpu():
    """``--model densenet201 --input 32 --classes 10 --phase frozen|finetune`` (dist_model_tf_dense.py
    phases 1 and 2): the softmax head, the frozen parameter counts and the per-phase metric name."""
    counts = {}
    for ph in ("frozen", "finetune"):
        r = _run(["--device", "cpu", "--model", "densenet201", "--input", "32", "--classes", "10",
                  "--phase", ph, "--batch", "2", "--steps", "1", "--warmup", "0", "--fit-steps", "0"])
        assert r.returncode == 0, r.stderr[-3000:]
        out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
        assert f"phase={ph}" in out["metric"] and "10-class" in out["metric"]
        assert out["config"]["input"] == [32, 32, 3] and out["config"]["classes"] == 10
        assert out["config"]["loss"].startswith("CategoricalCE")
        counts[ph] = out["config"]["trainable_params"]
    assert counts["frozen"] == 1920 * 10 + 10  # GAP(1920) -> Dense(10) only
    assert counts["frozen"] < counts["finetune"]


def test_bench_finetune_cuts_follow_the_reference():
    """``--phase finetune`` freezes ``layers[:fine_tune_at]`` with the reference's cut per backbone:
    VGG16 15 (block5 + head train: 7,079,937), MobileNetV2 100 in the 155-layer build (1,863,873)."""
    want = {"vgg16": 7079937, "mobilenetv2": 1863873}
    for model, n in want.items():
        r = _run(["--device", "cpu", "--model", model, "--phase", "finetune", "--batch", "2", "--steps", "1",
                  "--warmup", "0", "--fit-steps", "0"])
        assert r.returncode == 0, r.stderr[-3000:]
        out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
        assert out["config"]["trainable_params"] == n, (model, out["config"]["trainable_params"])
