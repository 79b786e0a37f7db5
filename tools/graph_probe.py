import torch, time
dev=torch.device('cuda',0)
x=torch.zeros(1,device=dev); y=torch.zeros(1<<20,device=dev)
for n in (1,13,26):
  for which in ('tiny','1M'):
    t = x if which=='tiny' else y
    s=torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3): 
            for i in range(n): t.add_(1)
    torch.cuda.current_stream().wait_stream(s)
    g=torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(n): t.add_(1)
    for _ in range(10): g.replay()
    torch.cuda.synchronize()
    e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200): g.replay()
    e1.record(); torch.cuda.synchronize()
    print(n, which, 'per graph %.1f us, per kernel %.2f us'%(e0.elapsed_time(e1)/200*1e3, e0.elapsed_time(e1)/200*1e3/n), flush=True)
