"""MI355X kernel ops (native HIP, gfx950) with PyTorch fp32 reference implementations."""
