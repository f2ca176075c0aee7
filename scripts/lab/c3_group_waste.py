import numpy as np, torch
from bitalosdb_amd import synth
from oracle import oracle as O
n=6000
v = synth.dict_values_gpu(n, 1024, device="cpu", seed=0xC3).numpy()
cost=[]; clen=[]; nel=[]
for r in v:
    s = O.snappy_encode(r.tobytes()); clen.append(len(s))
    p=0
    while s[p] >= 0x80: p+=1
    p+=1; e=0; ops=0
    while p < len(s):
        t=s[p]; ty=t&3
        if ty==0:
            x=t>>2
            if x<60: ln=x+1; p+=1
            else:
                nb=x-59; ln=int.from_bytes(s[p+1:p+1+nb],'little')+1; p+=1+nb
            p+=ln; ops+=(ln+15)//16
        else:
            if ty==1: ln=4+((t>>2)&7); off=((t&0xe0)<<3)|s[p+1]; p+=2
            elif ty==2: ln=1+(t>>2); off=int.from_bytes(s[p+1:p+3],'little'); p+=3
            else: ln=1+(t>>2); off=int.from_bytes(s[p+1:p+5],'little'); p+=5
            ops += (ln+15)//16 if off>=16 else -(-ln//off)
        e+=1
    nel.append(e); cost.append(85*e+10*ops)
cost=np.array(cost,float); clen=np.array(clen); nel=np.array(nel)
print("elements mean %.1f std %.1f; clen mean %.0f std %.0f; corr(clen,cost) %.2f corr(nel,cost) %.2f" % (nel.mean(), nel.std(), clen.mean(), clen.std(), np.corrcoef(clen,cost)[0,1], np.corrcoef(nel,cost)[0,1]))
def grp(c, B=18):
    m = len(c)//B*B
    return c[:m].reshape(-1,B).max(1).sum()/c[:m].sum()
print("natural order: sum(max)/sum = %.3f" % grp(cost))
for nb in (2,4,8):
    edges=np.quantile(clen, np.linspace(0,1,nb+1)[1:-1])
    b=np.searchsorted(edges, clen)
    order=np.concatenate([np.nonzero(b==k)[0] for k in range(nb)])
    print("%d clen buckets: %.3f" % (nb, grp(cost[order])))
print("sorted by cost: %.3f" % grp(np.sort(cost)))
print("sorted by clen: %.3f" % grp(cost[np.argsort(clen)]))
