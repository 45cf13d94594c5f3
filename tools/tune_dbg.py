import os, sys
sys.path.insert(0, "/root/repo")
os.environ["EXT_MPI_AMD_DEBUG_HIP"] = "1"; os.environ["EXT_MPI_AMD_DEBUG_TUNE"] = "1"
import torch, ext_mpi_collectives_amd as emac
R, n = 8, 4 << 20
s = [torch.rand(n, device="cuda") for _ in range(R)]; r = [torch.empty(n, device="cuda") for _ in range(R)]
h = emac.node_allreduce_init([t.data_ptr() for t in s], [t.data_ptr() for t in r], n, emac.FLOAT)
st = torch.cuda.Stream(); emac.set_stream(h, st.cuda_stream)
for k in range(7):
    try:
        emac.start(h); print("start", k, "ok", emac.handle_schedule(h), flush=True)
    except Exception as e:
        print("start", k, "failed", e, flush=True); break
st.synchronize()
print(torch.equal(r[0], r[7]))
