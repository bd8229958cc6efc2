import torch, torch.nn.functional as F, time
dev='cuda'
def t(fn, reps=10):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t0=time.perf_counter()
    for _ in range(reps): fn()
    torch.cuda.synchronize(); return (time.perf_counter()-t0)/reps*1e3
for (B,cin,cout,H) in [(64,256,128,256),(64,256,128,128),(64,512,256,64),(64,384,256,64),(64,1024,512,16)]:
    x=torch.randn(B,cin,H,H,device=dev); w=torch.randn(cout,cin,1,1,device=dev); b=torch.randn(cout,device=dev)
    dy=torch.randn(B,cout,H,H,device=dev)
    fl=2*B*H*H*cin*cout
    a=t(lambda: F.conv2d(x,w,b))
    c=t(lambda: torch.matmul(w[:,:,0,0], x.view(B,cin,-1)))
    d=t(lambda: torch.matmul(w[:,:,0,0].t(), dy.view(B,cout,-1)))
    print(f"B{B} {cin}->{cout} {H}^2: conv2d {a:.3f} ms {fl/a/1e9:.0f} TF/s | matmul fwd {c:.3f} ms {fl/c/1e9:.0f} | matmul bwd {d:.3f} ms {fl/d/1e9:.0f}", flush=True)
