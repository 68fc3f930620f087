import os, sys
REPO = os.environ["GRAFT_REPO_ROOT"]
for sub in ("uc-tcp-ip_amd", "oracle", "tests", ""):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np, torch, netcsum, oracle
rng = np.random.default_rng(5)
L, stride, n = 35, 36, 1025
bad_total = 0
for trial in range(int(os.environ.get("TRIALS", "20"))):
    for (k, tile, chunks) in ((7, -1, 0), (7, 2, 3), (7, 2, 2), (7, 2, 4), (7, 1, 2), (7, 1, 3), (7, 1, 4), (7, 4, 2), (7, 4, 3)):
        data = rng.integers(0, 256, size=n * stride + 128, dtype=np.uint8)
        d = torch.from_numpy(data).cuda()
        out = torch.zeros(n, dtype=torch.int16, device="cuda")
        netcsum.tune(netcsum.TUNE_KERNEL, k); netcsum.tune(netcsum.TUNE_TILE, tile); netcsum.tune(netcsum.TUNE_CHUNKS, chunks)
        netcsum.batch_strided(d, stride, L, None, 0, 0, n, out, 0)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint16)
        want = oracle.batch_strided(data, stride, L, None, 0, 0, n, 0)
        bad = np.nonzero(got != want)[0]
        if bad.size:
            bad_total += 1
            print(trial, k, tile, chunks, netcsum.last_launch(), bad.size, bad[:10].tolist(), flush=True)
print("bad runs", bad_total)
