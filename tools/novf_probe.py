import sys; sys.path.insert(0,'.')
import torch
from unsamflow_amd import _lib, ops
from unsamflow_amd.kernel_timer import site_launcher
lib=_lib.load(); dev=torch.device('cuda:0')
for (B,C,H,W) in [(16,32,64,208),(16,64,32,104)]:
    g=torch.Generator(device=dev).manual_seed(0)
    x=torch.rand(B,C,H,W,device=dev,generator=g); go=torch.randn(B,C,H,W,device=dev,generator=g)
    yy=torch.linspace(0,6.2832,H,device=dev).view(1,1,H,1); xx=torch.linspace(0,6.2832,W,device=dev).view(1,1,1,W)
    ph=torch.rand(B,2,1,1,device=dev,generator=g)*6.2832
    base=(torch.sin(2*xx+ph)+torch.cos(3*yy-ph)).contiguous()
    for name,fl in (("zero",torch.zeros_like(base)),("pm2",base),("pm8",(4*base).contiguous())):
        n=int(lib.usf_warp_bwd_workspace(B,H,W)); ws=torch.zeros(n,dtype=torch.uint8,device=dev)
        gx=torch.empty_like(x); gf=torch.empty(B,2,H,W,device=dev)
        for pad in (1,0):
            rc=lib.usf_warp_bwd_ex_f32(x.data_ptr(),fl.data_ptr(),2*H*W,go.data_ptr(),gx.data_ptr(),gf.data_ptr(),ws.data_ptr(),n,B,C,H,W,pad,torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            novf=int(ws[:4].view(torch.int32)[0])
            E=B*(H+1)*(W+1); cnt=ws[256:256+4*E].view(torch.int32)
            print((B,C,H,W),name,"border" if pad else "zeros","novf",novf,"of",B*H*W,"cnt hist",torch.bincount(cnt.long(),minlength=6)[:8].tolist(),flush=True)
