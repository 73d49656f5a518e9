import os, torch, dedloc_amd.ops
O = torch.ops.dedloc
torch.manual_seed(0)
for T in (4096, 131072):
    dy = (torch.rand(T, 1024, device='cuda') * 2 - 1).bfloat16()
    w = ((torch.rand(1024, 4096, device='cuda') * 2 - 1) * 0.05).bfloat16()
    f = torch.randn(T, 4096, device='cuda').bfloat16()
    for pol in ("mfma", "lib"):
        os.environ["DEDLOC_GEMM"] = pol
        db = torch.zeros(4096, device='cuda')
        df = O.gemm_dgelu(dy, w, f, db)
        ref = df.float().sum(0)
        print(T, pol, "rel(db, colsum(df))", ((db - ref).norm() / ref.norm()).item(), "db norm", db.norm().item())
