import os, sys, json
REPO = os.environ["GRAFT_REPO_ROOT"]
for sub in ("uc-tcp-ip_amd", "oracle", "tests", "tools", ""):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch, netcsum
from bench import SEED
from bench_configs import events_ms
dev = torch.device("cuda", 0); st = torch.cuda.current_stream(dev)
n, L = 1 << 20, 1500
pk = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
netcsum.fill(pk, n * L, SEED, 0)
v = pk[: n * L].view(n, L)
v[:, 0:12] = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], dtype=torch.uint8, device=dev)
flags = torch.zeros(n, dtype=torch.uint8, device=dev)
netcsum.tx_finalize_ipv4(pk, n, flags, stride=L, pkt_len=L); torch.cuda.synchronize()
r = {}
r["rx_flags"] = events_ms(lambda: netcsum.rx_validate_ipv4(pk, n, flags, stride=L, pkt_len=L, stream=st), st, reps=40)
r["tx_noflags"] = events_ms(lambda: netcsum.tx_finalize_ipv4(pk, n, None, stride=L, pkt_len=L, stream=st), st, reps=40)
r["tx_flags"] = events_ms(lambda: netcsum.tx_finalize_ipv4(pk, n, flags, stride=L, pkt_len=L, stream=st), st, reps=40)
r["rx_flags2"] = events_ms(lambda: netcsum.rx_validate_ipv4(pk, n, flags, stride=L, pkt_len=L, stream=st), st, reps=40)
print(json.dumps({k: round(x, 4) for k, x in r.items()}))
