import torch, sys
dev='cuda'
shapes=[(256,4096,768),(1024,2048,1536),(2560,2048,2048),(1024,2048,6144),(4096,4096,4096),(512,4096,2304)]
for M,N,K in shapes:
    A=torch.randn(M,K,device=dev); B=torch.randn(N,K,device=dev)
    C=torch.empty(M,N,device=dev)
    f=lambda: torch.mm(A,B.t(),out=C)
    for _ in range(3): f()
    torch.cuda.synchronize()
    g=torch.cuda.CUDAGraph()
    s=torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(20): f()
        g.replay()
        e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(3): g.replay()
        e1.record(s)
    e1.synchronize()
    us=e0.elapsed_time(e1)*1e3/60
    ref=(A.double()@B.double().t())
    err=((C.double()-ref).abs().max()/ref.abs().max()).item()
    print(f'torch.mm {M}x{N}x{K}: {us:8.1f} us {2*M*N*K/us/1e6:6.1f} TF err {err:.1e}', flush=True)
