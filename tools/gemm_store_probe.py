import sys; sys.path.insert(0,'.')
import ctypes as C, torch
from deephall_amd import _lib
lib=_lib.load()
def p(t): return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)
def run(v, rows, n, K, ldy, res=False, reps=20):
    rp=(rows+255)//256*256
    X=torch.randn(rp,K,device='cuda'); W=torch.randn(K,n,device='cuda')/16
    Wt=torch.zeros((n+255)//256*256,K,device='cuda'); Wt[:n]=W.t()
    Y=torch.empty(rp,n,device='cuda'); R=torch.randn(rp,n,device='cuda') if res else None
    s=C.c_void_p(torch.cuda.current_stream().cuda_stream)
    Wa,ldw=(Wt,K) if v>=100 else (W,n)
    args=(v,p(X),K,p(Wa),ldw,C.c_void_p(0),p(R),(n if ldy else 0),p(Y),ldy,rows,n,K,1,s)
    lib.dh_debug_gemm(*args); torch.cuda.synchronize()
    e0,e1=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): lib.dh_debug_gemm(*args)
    e1.record(); torch.cuda.synchronize()
    ms=e0.elapsed_time(e1)/reps
    return ms*1e3, 2*rows*n*K/(ms*1e-3)/1e12
for v in [9,105,106]:
    for (nm,n,res) in [("qkv",768,False),("d",256,False),("d_res",256,True)]:
        a=run(v,417792,n,256,n,res); b=run(v,417792,n,256,0,res)
        print(f"v{v} {nm}: full {a[0]:.0f}us {a[1]:.1f}TF   no-HBM-store {b[0]:.0f}us {b[1]:.1f}TF", flush=True)
