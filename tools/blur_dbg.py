import math, sys
import numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from oracle import blur as oblur, closed_form
from samplers_amd import _hip
from samplers_amd.operators import GaussianBlurOperator
cuda = torch.device('cuda')
for shape, batch, ydiv in (((2, 64, 256), 3, 3), ((1, 64, 256), 1, 1), ((1, 256, 256), 1, 1)):
    op = GaussianBlurOperator(shape, 9, 3.0).to(cuda)
    k1d = oblur.taps(9, 3.0)
    apply_np, adjoint_np = oblur.blur_ops(shape, k1d)
    lib = _hip.load_library(); desc = op.hip_descriptor(); n = math.prod(shape)
    P = lib.sp_rsq_partials(desc)
    torch.manual_seed(1)
    x, eps = torch.randn(batch, n), torch.randn(batch, n)
    y = torch.randn(batch // ydiv, n)
    a, k, gs = 0.3, math.sqrt(1 - 0.09), 400.0
    coefs = _hip.SpDpsCoefs(a, k, gs, 0.9, 0.2, 0.1, 0.05, 1e-9)
    xd, ed, yd = (t.to(cuda).contiguous() for t in (x, eps, y))
    v = torch.full_like(xd, float('nan')); part = torch.full((batch, P), float('nan'), device=cuda)
    _hip.check(lib.sp_dps_residual(desc, xd.data_ptr(), ed.data_ptr(), yd.data_ptr(), batch, ydiv, coefs, v.data_ptr(), part.data_ptr(), torch.cuda.current_stream().cuda_stream), 'r')
    v_ref, rsq_ref = closed_form.residual_pass(x.numpy(), eps.numpy(), y.numpy(), ydiv, a, k, gs, apply_np, adjoint_np)
    d = np.abs(v.cpu().numpy() - v_ref).reshape(batch, *shape)
    bad = d > 2e-5 * np.abs(v_ref).max()
    idx = np.argwhere(bad)
    print(shape, batch, 'bad', bad.sum(), 'rows', sorted(set(idx[:, 2].tolist()))[:40], 'cols', sorted(set(idx[:, 3].tolist()))[:20], 'rsq', part.sum(1).cpu().numpy(), rsq_ref)
