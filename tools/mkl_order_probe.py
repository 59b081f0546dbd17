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
def lca_sizes(K, M, N=1, col=0):
    """Leaf-set sizes of the smallest subtree joining each leaf pair (leaf K:
    the bias): x = 1, W_i = 2^40, W_j = -2^40, every other product 1 -- the
    ones absorbed into +-2^40 before the two cancel are the leaves of their
    joining subtree, so the result is (K + 1) - that subtree's size."""
    L = 2.0 ** 40
    def r(i, k):
        w = [1.0] * (K + 1); w[i] = L; w[k] = -L
        lin = torch.nn.Linear(K, M)
        with torch.no_grad():
            lin.weight.zero_(); lin.bias.zero_(); lin.weight[col] = torch.tensor(w[:K]); lin.bias[col] = w[K]
            return lin(torch.ones(N, K))[0, col].item()
    return [[0 if i == k else int(K + 1 - r(i, k)) for k in range(K + 1)] for i in range(K + 1)]

def tree32_check(trials=2000):
    """The 32 -> 32 1-row tree that lca_sizes(32, 32) gives, with its fma
    nodes (oracle/subdivide.py linear_seqfma, csrc/net_device.h), against
    torch on random inputs: returns the number of bitwise matches."""
    sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__file__), '..'))
    from oracle.subdivide import linear_seqfma
    lin = torch.nn.Linear(32, 32)
    ok = 0
    for t in range(trials):
        x = torch.randn(1, 32)
        with torch.no_grad():
            ok += bool(torch.equal(lin(x), linear_seqfma(x, lin)))
    return ok

if __name__=='__main__':
    if sys.argv[1:2] == ['tree32']:
        for row in lca_sizes(32, 32):
            print(row)
        print('tree32 bitwise matches:', tree32_check(), '/ 2000')
        sys.exit(0)
    for K,M,N in [(4,16,1),(8,16,1),(16,16,1),(16,2,1),(16,2,2),(16,2,15),(8,16,2),(16,16,3)]:
        t,fail=build_tree(K,M,N)
        print(K,M,N,t if t else ('FAIL',fail))
