import sys, time, numpy as np
import os; R=os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0,R); sys.path.insert(0,os.path.join(R,'tests'))
import lzbench_amd as L, oracle_lib as O
bad=0
for kind in ['text','json','random','binary']:
    d=L.datagen(kind, 1<<20, 7)
    for codec,chunk,lvl in [('lz4',65536,1),('snappy',65536,0),('lz4',131072,1),('snappy',262144,0),('lz4fast',65536,3)]:
        t=time.time(); p,cs=L.compress_chunks(d,codec,chunk,lvl); t1=time.time()-t
        op,ocs=O.compress_chunks(d,codec,chunk,lvl)
        ok=len(p)==len(op) and (p==op).all() and (cs==ocs).all()
        if not ok:
            bad+=1
            nz=np.nonzero(cs!=ocs)[0]
            print('MISMATCH',kind,codec,chunk,lvl,len(p),len(op),'first bad chunk',nz[:5], cs[nz[:3]], ocs[nz[:3]])
        r=L.decompress_chunks(op,ocs,len(d),codec,chunk)
        rt=(r==d).all()
        if not rt: bad+=1; print('RT FAIL',kind,codec,chunk, np.nonzero(r!=d)[0][:5])
        print(kind,codec,chunk,lvl,'exact',ok,'rt',rt,'%.3fs'%t1, flush=True)
print('BAD',bad)
