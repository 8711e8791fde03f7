import math, torch
from stableavatar_amd import ops
dev="cuda"; torch.manual_seed(0)
for (M,N,K) in [(4032,1536,1536),(1024,512,256)]:
    x=torch.randn(M,K,device=dev).bfloat16(); w=(torch.randn(N,K,device=dev)/math.sqrt(K)).bfloat16(); b=torch.randn(N,device=dev)
    ref=x.float()@w.float().t()+b
    for rep in range(3):
        y=ops.linear(x,w,b,ops.EPI_F32)
        bad=((y-ref).abs()>1e-2*(ref.abs()+1)).nonzero()
        print(M,N,K,"rep",rep,"bad",bad.shape[0], flush=True)
        if bad.shape[0]:
            r=bad[:,0]; c=bad[:,1]
            print(" tiles", sorted(set(((r//256)*100+(c//256)).tolist()))[:40])
            print(" rows%256", torch.bincount(r%256,minlength=256).nonzero().flatten()[:40].tolist())
            print(" cols%256", torch.bincount(c%256,minlength=256).nonzero().flatten()[:40].tolist())
            print(" sample", [(int(a),int(bb),float(y[a,bb]),float(ref[a,bb])) for a,bb in bad[:5].tolist()])
