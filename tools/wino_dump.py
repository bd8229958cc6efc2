"""Dump Winograd-tile outputs for fixed inputs, to compare two library builds bit for bit:

    SAMPLERS_HIP_LIB=a.so python tools/wino_dump.py out_a.pt
    SAMPLERS_HIP_LIB=b.so python tools/wino_dump.py out_b.pt
    python tools/wino_dump.py --compare out_a.pt out_b.pt
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

SHAPES = [(4, 128, 128, 64, 64), (3, 256, 128, 16, 16), (5, 512, 256, 8, 8), (2, 64, 64, 32, 96)]


def dump(path):
    from samplers_amd import _hip

    lib = _hip.load_library()
    st = torch.cuda.current_stream().cuda_stream
    out = {}
    for shape in SHAPES:
        n, cin, cout, h, w = shape
        g = torch.Generator().manual_seed(sum(shape))
        x = torch.randn(n, cin, h, w, generator=g).cuda()
        wt = (torch.randn(cout, cin, 3, 3, generator=g) * (cin * 9) ** -0.5).cuda()
        b = torch.randn(cout, generator=g).cuda()
        res = torch.randn(n, cout, h, w, generator=g).cuda()
        dy = torch.randn(n, cout, h, w, generator=g).cuda()
        up = torch.empty(lib.sp_wino3x3_packed_size(cin, cout), device="cuda")
        uv = torch.empty_like(up)
        _hip.check(lib.sp_wino3x3_pack(wt.data_ptr(), cout, cin, 0, up.data_ptr(), st), "pack")
        _hip.check(lib.sp_wino3x3_pack(wt.data_ptr(), cout, cin, 1, uv.data_ptr(), st), "pack vjp")
        y = torch.empty(n, cout, h, w, device="cuda")
        yr = torch.empty_like(y)
        dx = torch.empty_like(x)
        _hip.check(lib.sp_wino3x3_fwd(x.data_ptr(), up.data_ptr(), b.data_ptr(), n, cin, cout, h, w,
                                      y.data_ptr(), st), "fwd")
        _hip.check(lib.sp_wino3x3_fwd_res(x.data_ptr(), up.data_ptr(), b.data_ptr(), res.data_ptr(), n,
                                          cin, cout, h, w, yr.data_ptr(), st), "fwd_res")
        _hip.check(lib.sp_wino3x3_bwd_input(dy.data_ptr(), uv.data_ptr(), n, cin, cout, h, w,
                                            dx.data_ptr(), st), "bwd")
        torch.cuda.synchronize()
        out[str(shape)] = (y.cpu(), yr.cpu(), dx.cpu())
    torch.save(out, path)


def compare(a, b):
    da, db = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    ok = True
    for k in da:
        for name, ta, tb in zip(("fwd", "fwd_res", "bwd"), da[k], db[k]):
            same = torch.equal(ta, tb)
            ok &= same
            print(k, name, "bit-identical" if same else f"max diff {(ta - tb).abs().max().item():.3e}")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        dump(sys.argv[1])
