import sys, time, json
sys.path[:0]=['/root/repo/reductionist-rs_amd','/root/repo']
import os
sys.path[:0]=[os.environ.get('GRAFT_REPO_ROOT','.')+'/reductionist-rs_amd', os.environ.get('GRAFT_REPO_ROOT','.')]
import torch
from reductionist_amd import Engine, _abi
eng=Engine([0]); ws=eng.workspace(0)
n=int(sys.argv[1]); mib=int(sys.argv[2])
g=torch.Generator(device='cuda'); g.manual_seed(1)
chunks=[torch.randint(0,16,(mib<<18,),dtype=torch.int32,device='cuda',generator=g).float() for _ in range(min(n,64))]
ptrs=[chunks[i%len(chunks)].data_ptr() for i in range(n)]
creq=_abi.CRequest("sum","float32",filters=[{"id":"shuffle","element_size":4}])
out=torch.zeros(n,dtype=torch.float32,device='cuda'); cnt=torch.zeros(n,dtype=torch.int64,device='cuda'); st=torch.zeros(n,dtype=torch.int32,device='cuda')
s=torch.cuda.current_stream()
for k in range(3):
    t0=time.time()
    ws.execute_batch_device(creq, ptrs, mib<<20, out.data_ptr(), cnt.data_ptr(), st.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    rec = {"n":n,"mib":mib,"k":k,"s":round(time.time()-t0,4),"cnt0":int(cnt[0]),"st":int(st.abs().sum())}
    lib = _abi.lib()
    if hasattr(lib, "rdx_probe_read_f32"):
        import ctypes as C
        buf = (C.c_uint64 * (8 * 8192))()
        lib.rdx_probe_read_f32(buf, 8 * 8192)
        nwg = int(sys.argv[3]) if len(sys.argv) > 3 else 64
        rec["wg"] = [[i, (buf[8*i+1]-buf[8*i])//100, buf[8*i+2] > 0, buf[8*i+5], buf[8*i+6] >> 32, buf[8*i+6] & 0xffffffff] for i in range(nwg)]
    print(json.dumps(rec), flush=True)
