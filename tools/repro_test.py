"""Call one GPU test function N times in one process and count failures (flake hunting).

usage: python tools/repro_test.py tests/test_fused_gpu.py test_a,test_b N
"""
import gc
import importlib.util
import os
import sys
import traceback

sys.path.insert(0, ".")


def main():
    path, names, n = sys.argv[1], sys.argv[2].split(","), int(sys.argv[3])
    spec = importlib.util.spec_from_file_location("t", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    keep = os.environ.get("REPRO_KEEP", "")
    if keep:
        from idc_models_amd.engine import model as model_mod
        from idc_models_amd.engine import arena as arena_mod
        KEPT = []
        if "model" in keep:
            orig = model_mod.Model.__init__

            def init(self, *a, **k):
                orig(self, *a, **k)
                KEPT.append(self)
            model_mod.Model.__init__ = init
        if "arena" in keep:
            orig_a = arena_mod.ParamArena.__init__

            def ainit(self, *a, **k):
                orig_a(self, *a, **k)
                KEPT.append((self.data, self.grad))
            arena_mod.ParamArena.__init__ = ainit
        if "net" in keep:
            orig_n = model_mod.Model.__init__

            def ninit(self, net, *a, **k):
                orig_n(self, net, *a, **k)
                KEPT.append([t for t in net.state_dict().values()] + list(net.parameters()))
            model_mod.Model.__init__ = ninit
    if os.environ.get("REPRO_SAVEALL") == "1":
        gc.set_debug(gc.DEBUG_SAVEALL)  # collected cycles are kept in gc.garbage, never freed
    fails = 0
    for i in range(n):
        for name in names:
            try:
                getattr(mod, name)()
                if os.environ.get("REPRO_GC") == "1":
                    gc.collect()
                print(f"run {i} {name}: ok", flush=True)
            except AssertionError:
                fails += 1
                print(f"run {i} {name}: FAIL {traceback.format_exc().splitlines()[-1][:300]}", flush=True)
    print(f"{fails}/{n * len(names)} failed")
    if os.environ.get("REPRO_SAVEALL") == "1":
        import collections
        import torch
        kinds = collections.Counter(type(o).__name__ for o in gc.garbage)
        print("garbage types:", kinds.most_common(25))
        cuda = collections.Counter(tuple(o.shape) for o in gc.garbage
                                   if isinstance(o, torch.Tensor) and o.is_cuda)
        print("cuda tensors in garbage:", sum(cuda.values()), cuda.most_common(10))


if __name__ == "__main__":
    main()
