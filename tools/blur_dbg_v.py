"""Debug: the streaming blur kernel built with -DSP_BLUR_DBG=1 stores the vertical adjoint V
of S = gs (y - A x0) (before the horizontal adjoint); compare with torch on the host."""
import math, sys
import numpy as np, torch, torch.nn.functional as F
sys.path.insert(0, '.')
from oracle import blur as oblur
from samplers_amd import _hip
from samplers_amd.operators import GaussianBlurOperator
cuda = torch.device('cuda')
shape, batch = (1, 64, 256), 1
op = GaussianBlurOperator(shape, 9, 3.0).to(cuda)
k1d = oblur.taps(9, 3.0)
lib = _hip.load_library(); desc = op.hip_descriptor(); n = math.prod(shape)
P = lib.sp_rsq_partials(desc)
torch.manual_seed(1)
x, eps = torch.randn(batch, n), torch.randn(batch, n)
y = torch.randn(batch, n)
a, k, gs = 0.3, math.sqrt(1 - 0.09), 400.0
coefs = _hip.SpDpsCoefs(a, k, gs, 0.9, 0.2, 0.1, 0.05, 1e-9)
xd, ed, yd = (t.to(cuda).contiguous() for t in (x, eps, y))
v = torch.full_like(xd, float('nan')); part = torch.full((batch, P), float('nan'), device=cuda)
_hip.check(lib.sp_dps_residual(desc, xd.data_ptr(), ed.data_ptr(), yd.data_ptr(), batch, 1, coefs, v.data_ptr(), part.data_ptr(), torch.cuda.current_stream().cuda_stream), 'r')
x0 = ((x.double() - k * eps.double()) / a).reshape(batch, *shape)
S = gs * (y.double().reshape(batch, *shape) - oblur.blur(x0, k1d))
kk = torch.from_numpy(k1d.astype(np.float64))
z = torch.zeros_like(S, requires_grad=True)
with torch.enable_grad():
    pad = F.pad(z.reshape(-1, 1, shape[1], shape[2]), (0, 0, 4, 4), mode='reflect')
    out = F.conv2d(pad, kk.view(1, 1, 9, 1))
    (V,) = torch.autograd.grad(out, z, S.reshape(out.shape))
V = V.reshape(shape[1], shape[2]).numpy()
got = v.cpu().double().reshape(shape[1], shape[2]).numpy()
d = np.abs(got - V); bad = d > 1e-4 * np.abs(V).max()
idx = np.argwhere(bad)
print('V bad', bad.sum(), 'rows', sorted(set(idx[:, 0].tolist()))[:40], 'cols', sorted(set(idx[:, 1].tolist()))[:40])
