import os, sys, torch
os.environ["IDC_AUTOTUNE"]="0"; os.environ["IDC_DETERMINISTIC"]="1"
sys.path.insert(0, ".")
from idc_models_amd.engine import Model, RMSprop
from idc_models_amd.models import build_model
from idc_models_amd.parallel import OneDeviceStrategy
from idc_models_amd.runtime.program import FusedProgram
m = Model(build_model("vgg16", None, 1, seed=7), OneDeviceStrategy("cuda:0"))
m.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
g = torch.Generator().manual_seed(3)
x = torch.randint(0, 256, (9, 50, 50, 3), generator=g, dtype=torch.uint8)
y = torch.randint(0, 2, (9,), generator=g)
res = []
for w in (1.0, 1.5):
    p = FusedProgram(m, 9, True, torch.uint8, grad_weight=w, use_graphs=False)
    m.impl._stage_inputs(p, x, y)
    p.run_segment("fwd"); p.run_segment("bwd")
    torch.cuda.current_stream().wait_stream(p.stream); torch.cuda.synchronize()
    res.append(m.arena.grad.clone().double())
print("ratio", float(res[1].norm() / res[0].norm()), "rel", float((res[1] - 1.5 * res[0]).norm() / res[1].norm()))
