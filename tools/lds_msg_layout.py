import itertools, random
SIG=[[0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15],[14,10,4,8,9,15,13,6,1,12,0,2,11,7,5,3],[11,8,12,0,5,2,15,13,10,14,3,6,7,1,9,4],[7,9,3,1,13,12,11,14,2,6,5,10,4,0,15,8],[9,0,5,7,2,4,10,15,14,1,11,12,6,8,3,13],[2,12,6,10,0,11,8,3,4,13,7,5,15,14,1,9],[12,5,1,15,14,13,4,10,0,7,6,3,9,2,8,11],[13,11,7,14,12,1,3,9,5,0,15,4,8,6,2,10],[6,15,14,9,11,3,0,8,12,2,13,7,1,4,10,5],[10,2,8,4,7,6,1,5,15,11,9,14,3,12,13,0]]
SIG=SIG+SIG[:2]
reads=[]
for r in range(12):
    s=SIG[r]
    reads.append([s[2*j] for j in range(4)]); reads.append([s[2*j+1] for j in range(4)])
    reads.append([s[8+2*j] for j in range(4)]); reads.append([s[9+2*j] for j in range(4)])
def cost(pair):  # pair(q,w) -> bank pair 0..31 ; group = quads 0..7
    tot=0
    for W in reads:
        cnt=[0]*32
        for q in range(8):
            for w in W: cnt[pair(q,w)%32]+=1
        tot+=max(cnt)
    return tot
print("baseline stride16:", cost(lambda q,w: 16*q+w))
for S in range(16,40):
    print("stride",S, cost(lambda q,w,S=S: S*q+w))
random.seed(1)
def cost_perm(P):
    return cost(lambda q,w: 16*(q&1)+P[q][w])
best=None
for trial in range(6):
    P=[list(range(16)) for _ in range(8)]
    for p in P: random.shuffle(p)
    c=cost_perm(P); T=2.0
    for it in range(40000):
        q=random.randrange(8); a,b=random.sample(range(16),2)
        P[q][a],P[q][b]=P[q][b],P[q][a]
        c2=cost_perm(P)
        if c2<=c or random.random()<pow(2.718,(c-c2)/T): c=c2
        else: P[q][a],P[q][b]=P[q][b],P[q][a]
        T=max(0.05,T*0.9998)
    print("trial",trial,c)
    if best is None or c<best[0]: best=(c,[p[:] for p in P])
print(best)
