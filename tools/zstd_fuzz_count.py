"""tools/zstd_fuzz_count.py -- corrupted zstd frames: how often the GPU decoder and the reference
ZSTD_decompressDCtx disagree on accepting (LZH_LIB=build/exp/<dbg> with -DLZH_ZSTD_DEBUG=1 gives line codes)"""
import sys, numpy as np
sys.path.insert(0,'tests'); sys.path.insert(0,'.')
import torch, oracle_lib as O, lzbench_amd as L
from test_gpu_zstd import _corrupt, gpu_decode
torch.cuda.set_device(0)
for kind in ("text","json","mixed"):
    chunk=32768; rng=np.random.default_rng(5+len(kind))
    data=L.datagen(kind,8*chunk,31)
    packed,cs=O.compress_chunks(data,"zstd",chunk,1)
    offs=np.concatenate([[0],np.cumsum(cs)]).astype(np.int64)
    valid=[packed[offs[i]:offs[i+1]].tobytes() for i in range(len(cs))]
    streams=[]
    while len(streams)<2048:
        s=_corrupt(rng,valid[int(rng.integers(0,len(valid)))])
        if 0<len(s)!=chunk: streams.append(s)
    st,out=gpu_decode(torch,np.frombuffer(b"".join(streams),np.uint8),[len(s) for s in streams],len(streams)*chunk,chunk)
    R=O.ref(); gpu_only=ref_only=same=0; ex=[]
    for i,s in enumerate(streams):
        src=np.frombuffer(s,np.uint8).copy(); dst=np.zeros(chunk+64,np.uint8)
        r=R.ref_zstd_decompress(src.ctypes.data,len(s),dst.ctypes.data,chunk)
        g=st[i]==chunk; rr=r==chunk
        if g and not rr: gpu_only+=1
        elif rr and not g: ref_only+=1; ex.append((i,int(st[i]),int(r)))
        else: same+=1
    from collections import Counter
    print(kind,"same",same,"gpu-only-accept",gpu_only,"ref-only-accept",ref_only,Counter(e[1] for e in ex).most_common(8),flush=True)
