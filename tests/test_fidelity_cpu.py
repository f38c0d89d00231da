"""utils/fidelity.py: the per-parameter fidelity bound the GPU tests use (CPU, synthetic gradients)
and secure aggregation's per-segment range helper (CPU path)."""
import torch

from idc_models_amd.utils import fidelity as fd


class _Arena:
    """Flat-gradient view by parameter index, like engine.arena.ParamArena."""

    def __init__(self, shapes):
        self.shapes = shapes
        self.offs = []
        o = 0
        for s in shapes:
            self.offs.append(o)
            o += int(torch.Size(s).numel())
        self.n = o

    def view(self, flat, i):
        n = int(torch.Size(self.shapes[i]).numel())
        return flat[self.offs[i]:self.offs[i] + n].view(self.shapes[i])


def _setup(seed=0):
    g = torch.Generator().manual_seed(seed)
    shapes = [(64,), (3, 3, 8, 16), (16,), (1,)]
    g32 = [torch.randn(s, generator=g, dtype=torch.float64) for s in shapes]
    g32[0] *= 1e-6  # an (almost) invariant direction: per-element RMS << the median
    noise = [0.3 * torch.randn(s, generator=g, dtype=torch.float64) * t.abs().mean().clamp_min(1e-3)
             for s, t in zip(shapes, g32)]
    g16 = [a + b for a, b in zip(g32, noise)]
    return _Arena(shapes), g32, g16, g


def test_fused_like_autocast_passes():
    ar, g32, g16, g = _setup()
    fused = torch.cat([(a + 0.9 * (b - a)).reshape(-1) for a, b in zip(g32, g16)]).float()
    assert fd.grad_failures(ar, fused, g32, g16) == []


def test_wrong_magnitude_fails_even_with_perfect_direction():
    ar, g32, g16, g = _setup()
    parts = [a.clone() for a in g32]
    parts[1] = 3.0 * parts[1]  # right direction, 3x too large: cosine 1, relative error 2
    bad = fd.grad_failures(ar, torch.cat([p.reshape(-1) for p in parts]).float(), g32, g16)
    assert [b["param"] for b in bad] == [1]


def test_invariant_direction_is_bounded_on_the_gradient_scale():
    ar, g32, g16, g = _setup()
    parts = [a.clone() for a in g32]
    med = sorted(float(t.norm()) / t.numel() ** 0.5 for t in g32)[len(g32) // 2]
    parts[0] = torch.full_like(parts[0], 0.5 * med)   # noise on the invariant param: allowed
    assert fd.grad_failures(ar, torch.cat([p.reshape(-1) for p in parts]).float(), g32, g16) == []
    parts[0] = torch.full_like(parts[0], 5.0 * med)   # blown up: flagged
    bad = fd.grad_failures(ar, torch.cat([p.reshape(-1) for p in parts]).float(), g32, g16)
    assert bad and bad[0]["param"] == 0 and bad[0]["invariant"]


def test_segment_absmax_cpu():
    from idc_models_amd.fed.secagg import segment_absmax, segment_ends
    sizes = [3, 1, 5]
    v1 = torch.tensor([1., -4., 2., 0.5, 3., -7., 1., 0., 2.])
    v2 = torch.tensor([-5., 1., 0., -0.25, 1., 1., 9., 0., -1.])
    got = segment_absmax([v1, v2], segment_ends(sizes), 3, "cpu")
    assert torch.equal(got, torch.tensor([5., 0.5, 9.]))


def test_one_noise_draw_past_the_soft_bound_is_tolerated_many_are_not():
    g = torch.Generator().manual_seed(5)
    shapes = [(32,)] * 10
    ar = _Arena(shapes)
    g32 = [torch.randn(s, generator=g, dtype=torch.float64) for s in shapes]
    e = [torch.randn(s, generator=g, dtype=torch.float64) for s in shapes]
    g16 = [a + 0.2 * a.norm() / b.norm() * b for a, b in zip(g32, e)]  # autocast: rel 0.2 each

    def fused(scales):  # rel(fused) = scale * 0.2 along the same noise direction
        return torch.cat([(a + s * (b - a)).reshape(-1) for a, b, s in zip(g32, g16, scales)]).float()
    assert fd.grad_failures(ar, fused([1.8] + [1.0] * 9), g32, g16) == []        # one soft draw
    assert len(fd.grad_failures(ar, fused([1.8] * 3 + [1.0] * 7), g32, g16)) == 3  # several: fail
    assert len(fd.grad_failures(ar, fused([2.3] + [1.0] * 9), g32, g16)) == 1     # past the hard bound
