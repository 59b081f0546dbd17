"""Probe the summation tree torch.nn.Linear (x86 MKL sgemm) uses for a given
(K inputs, M outputs, N rows): with W = 1, a product pair (j, l) = 2^-24 each
and p_i = 1, the result differs from 1 iff j and l are added before meeting i.
Used to derive oracle/subdivide.py::linear_seqfma (CPU only; no GPU)."""
import sys; pass
import torch, itertools
torch.set_num_threads(1)
d=2.0**-24
def run(K,M,N,vals,bvals,row=0,col=0):
    lin=torch.nn.Linear(K,M)
    with torch.no_grad():
        lin.weight.fill_(1.0); lin.bias.fill_(0.0); lin.bias[col]=bvals
        x=torch.zeros(N,K); x[row]=torch.tensor(vals)
        return lin(x)[row,col].item()
def R(K,M,N,i,j,l,row=0,col=0):
    v=[0.0]*(K+1); v[i]=1.0; v[j]=d; v[l]=d
    return run(K,M,N,v[:K],v[K],row,col)!=1.0
def build_tree(K,M,N,row=0,col=0):
    nodes={t:t for t in range(K+1)}  # rep -> tree
    while len(nodes)>1:
        reps=list(nodes)
        merged=False
        for a,b in itertools.combinations(reps,2):
            others=[i for i in reps if i not in (a,b)]
            if all(R(K,M,N,i,a,b,row,col) for i in others):
                nodes[a]=(nodes[a],nodes[b]); del nodes[b]; merged=True; break
        if not merged:
            return None, nodes
    return list(nodes.values())[0], None
if __name__=='__main__':
    for K,M,N in [(4,16,1),(8,16,1),(16,16,1),(16,2,1),(16,2,2),(16,2,15),(8,16,2),(16,16,3)]:
        t,fail=build_tree(K,M,N)
        print(K,M,N,t if t else ('FAIL',fail))
