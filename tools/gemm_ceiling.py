"""Library ceiling for VGG16's convolutions: hipBLASLt (torch.matmul, bf16) on plain GEMMs of the
same M x K x N as each VGG16 3x3 conv at 50x50, batch 256 (implicit GEMM: M = N*H*W pixels,
K = 9*Cin, N = Cout).  A plain GEMM has no im2col gather and no padding, so it bounds what an
implicit-GEMM kernel on the same shape can reach; compare with the conv_big per-layer times of
profiles/vgg16_bs256_kernels.md.

    python tools/gemm_ceiling.py [--reps 20]
"""
import argparse

import torch

LAYERS = [  # (name, H, Cin, Cout)
    ("b1c2", 50, 64, 64), ("b2c1", 25, 64, 128), ("b2c2", 25, 128, 128),
    ("b3c1", 12, 128, 256), ("b3c2", 12, 256, 256), ("b4c1", 6, 256, 512), ("b4c2", 6, 512, 512),
    ("b5c1", 3, 512, 512),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    print("| layer | M | K | N | GFLOP | hipBLASLt us | TFLOP/s | % of 2.5 PF |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|")
    for name, H, cin, cout in LAYERS:
        M, K, N = a.batch * H * H, 9 * cin, cout
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            torch.matmul(x, w)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            torch.matmul(x, w)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) / a.reps * 1e3
        gf = 2.0 * M * K * N / 1e9
        tf = gf / us * 1e3  # GFLOP/us = PFLOP/s
        print(f"| {name} | {M} | {K} | {N} | {gf:.1f} | {us:.1f} | {tf:.0f} | {100 * tf / 2500:.0f}% |", flush=True)
        del x, w


if __name__ == "__main__":
    main()
