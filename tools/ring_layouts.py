"""Device-resident NIC-ring layouts for the packet rows of DESIGN.md §9 (GPU box only; imported by
tools/run_config.py and tools/ring_probe.py).

The reference's receive buffers are fixed-size pool buffers, one NET_BUF per frame
(/root/reference/Cfg/Template/net_dev_cfg.c:146-149: 1518-B large buffers, 4-B alignment, so a
1520-B slot; Source/net_buf.h:595-598), the frame length coming per frame from the driver
(IF/net_if.c:6593). Two ways a driver hands such a ring over:
  strided        base = slot 0 + 14 (the IPv4 header after the Ethernet header), stride = slot,
                 pkt_len = the bytes present per slot (slot - 14): every frame's extent is parsed
                 from its own IPv4 header;
  offset/length  off[i] = slot i + 14, len[i] = the frame length the driver reports minus the
                 Ethernet header (a frame is at least 60 B, so a 40-B datagram has 46 B).

mixed_ring(): datagrams of 40 / 576 / 1500 B at 7 : 4 : 1 (TCP ACKs, default-MSS UDP datagrams,
full-size TCP segments) in random order. Byte values from the device splitmix64 fill; the first 40
bytes of every frame are an IPv4 header (20 B, total length = the datagram size) and a TCP header
(data offset 5) or a UDP header (length = size - 20, checksum field left for Tx to compute)."""
import numpy as np

SIZES = np.array([40, 576, 1500], np.int64)
WEIGHTS = np.array([7, 4, 1], np.float64) / 12.0


def ring_sizes(n, seed=11):
    return SIZES[np.random.default_rng(seed).choice(3, size=n, p=WEIGHTS)]


def headers(sizes, seed=12):
    """(n, 40) uint8: IPv4 header + TCP header (40-B and 1500-B datagrams) or UDP header + 12 payload
    bytes (576-B datagrams), checksum fields 0 (Tx computes them)."""
    n = len(sizes)
    rng = np.random.default_rng(seed)
    h = rng.integers(0, 256, size=(n, 40), dtype=np.uint8)
    udp = sizes == 576
    h[:, 0] = 0x45
    h[:, 1] = 0
    h[:, 2] = (sizes >> 8) & 0xFF
    h[:, 3] = sizes & 0xFF
    h[:, 6] = 0x40                                   # DF, offset 0
    h[:, 7] = 0
    h[:, 8] = 64
    h[:, 9] = np.where(udp, 17, 6)
    h[:, 10:12] = 0
    h[:, 32] = np.where(udp, h[:, 32], 0x50)         # TCP data offset 5 (byte 12 of the TCP header)
    ulen = sizes - 20
    h[:, 24] = np.where(udp, (ulen >> 8) & 0xFF, h[:, 24])
    h[:, 25] = np.where(udp, ulen & 0xFF, h[:, 25])
    h[:, 26] = np.where(udp, 0, h[:, 26])            # UDP checksum (20 + 6) / TCP sequence bytes
    h[:, 27] = np.where(udp, 0, h[:, 27])
    h[:, 36:38] = np.where(udp[:, None], h[:, 36:38], 0)   # TCP checksum field (20 + 16)
    return h


def mixed_ring(torch, netcsum, dev, n, slot=1520, lead=14, seed=0x5EED0001, sizes=None):
    """-> dict(buf, base (slot 0 + lead), sizes, off / lens (device, the offset/length form: offsets
    into buf), present,
    datagram_bytes). The whole ring is one device allocation of n * slot bytes (+ 256)."""
    sizes = ring_sizes(n) if sizes is None else np.asarray(sizes, np.int64)
    buf = torch.empty(n * slot + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(buf, n * slot, seed, 0)
    buf[: n * slot].view(n, slot)[:, lead:lead + 40] = torch.from_numpy(headers(sizes)).to(dev)
    off = (np.arange(n, dtype=np.uint64) * np.uint64(slot) + np.uint64(lead)).astype(np.uint64)   # into buf
    lens = np.maximum(sizes, 46).astype(np.uint16)
    return {"buf": buf, "base": buf[lead:], "sizes": sizes, "present": slot - lead,
            "off": torch.from_numpy(off.view(np.int64)).to(dev),
            "lens": torch.from_numpy(lens.view(np.int16)).to(dev),
            "datagram_bytes": int(sizes.sum()), "slot": slot, "lead": lead}


def uniform_ring(torch, netcsum, dev, n, slot, lead, size=1500):
    """1500-B IPv4/TCP datagrams, one per slot at +lead (the template and 2-KiB layouts)."""
    return mixed_ring(torch, netcsum, dev, n, slot, lead, sizes=np.full(n, size, np.int64))
