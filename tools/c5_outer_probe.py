"""C5 outer objective (make_lenet, S = 256, M = 500 + a 128-row batch): d/du
and the parameter gradient of one world-1 plan against the sum of 8 sample
shards of 32 (psvi_outer_elbo_grad_coef with the global coefficients), with
the conv towers on the VALU kernels and on MFMA -- identical parameters, so
the two decompositions differ by fp32 summation order only."""
import os, sys, torch, numpy as np
ROOT="/root/repo" if os.path.exists("/root/repo") else os.environ["GRAFT_REPO_ROOT"]
sys.path[:0]=[os.path.join(ROOT,"blackbox-coresets-vi_amd"), os.path.join(ROOT,"tests"), os.path.join(ROOT,"oracle")]
from golden_util import l2rel
from psvi.runtime import InnerLoopPlan, randn_, _lib
from psvi.runtime.sharded import local_eps, sample_split, outer_coefficients, pack_coef
LENET=[(25,6),(150,16),(400,120),(120,84),(84,10)]
S,M,Nx=256,500,128
g=torch.Generator().manual_seed(3)
u=torch.randn(M,784,generator=g); xb=torch.randn(Nx,784,generator=g)
z=torch.randint(0,10,(M+Nx,),generator=g).int()
from psvi.models import make_lenet
torch.manual_seed(0)
p=torch.nn.utils.parameters_to_vector(make_lenet(mc_samples=S,init_sd=0.05).parameters()).detach().cuda()
x_all=torch.cat([u,xb]).cuda().contiguous(); z_all=z.cuda(); w_all=torch.cat([torch.full((M,),120.0),torch.full((Nx,),60000.0/Nx)]).cuda()
lib=_lib.load()
for valu in (1,0):
    lib.psvi_debug_set(16,valu)
    one=InnerLoopPlan("lenet",LENET,S,M+Nx)
    e=torch.empty(one.eps_count,device="cuda"); randn_(e,5)
    o1=one.outer_elbo_grad(M,x_all,z_all,w_all,e,p,sample_stats=True)
    terms=o1["samples"][:,:3].contiguous()
    loss,cp,cd,ck=outer_coefficients(terms)
    gu8=torch.zeros_like(o1["grad_u"]); g8=torch.zeros_like(o1["grad"])
    for r,(off,cnt) in enumerate(sample_split(S,8)):
        pl=InnerLoopPlan("lenet",LENET,cnt,M+Nx)
        el=local_eps("lenet",LENET,S,off,cnt,e)
        coef=pack_coef(cp,cd,ck,off,cnt).cuda()
        gg=pl.outer_grad_coef(M,x_all,z_all,w_all,el,p,coef)
        gu8+=gg["grad_u"]; g8+=gg["grad"]
    a=o1["grad_u"].cpu().numpy().reshape(M,-1); b=gu8.cpu().numpy().reshape(M,-1)
    err=np.linalg.norm(a-b,axis=1)/np.linalg.norm(a,axis=1)
    print(f"valu={valu}: outer grad_u w1 vs 8x32: l2rel {l2rel(b,a):.2e} rows>1e-4 {(err>1e-4).sum()} median {np.median(err):.2e}; grad {l2rel(g8.cpu().numpy(),o1['grad'].cpu().numpy()):.2e}",flush=True)
