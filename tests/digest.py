"""Order-free digest of HM_KEY cells on the device: tests/conftest.py's
cells_digest (the C oracle's, tests/golden/make_bigdigest.py) in torch int64
arithmetic.  Shared by tests/test_gpu_fullsize.py and tools/bench_stream.py."""

M29 = (1 << 29) - 1
_U = (1 << 64) - 1


def _s64(v):
    return v - (1 << 64) if v >= 1 << 63 else v


def device_digest(torch, keys, counts):
    """tests/conftest.py cells_digest of HM_KEY cells, on the device (int64
    arithmetic wraps like the uint64 original; right shifts made logical)."""
    return device_cells_digest(torch, keys >> 58, (keys >> 29) & M29, keys & M29, counts)


def device_cells_digest(torch, z, r, c, counts):
    """cells_digest of (zoom, row, col, count) int64 CUDA tensors."""

    def lsr(x, k):
        return (x >> k) & ((1 << (64 - k)) - 1)

    x = (z * _s64(0x9E3779B97F4A7C15)) ^ r
    x = (x * _s64(0xBF58476D1CE4E5B9)) ^ c
    x = (x * _s64(0x94D049BB133111EB)) ^ counts
    x = x ^ lsr(x, 31)
    x = x * _s64(0xD6E8FEB86659FD93)
    x = x ^ lsr(x, 32)
    s = int(x.sum().item()) & _U
    while x.numel() > 1:
        h = x.numel() // 2
        y = x[:h] ^ x[h:2 * h]
        x = torch.cat([y, x[2 * h:]]) if x.numel() & 1 else y
    xr = (int(x[0].item()) & _U) if x.numel() else 0
    return [int(z.numel()), int(counts.sum().item()), s, xr]
