"""The drop-in boundary, checked by a compiler and a C caller (no GPU needed):

* the checksum and CRC prototypes of include/netcsum_mi355x.h and of the in-stack stand-in
  tests/instack/net_util.h equal the reference's Source/net_util.h:422-450 token for token, and every NET_BUF field the chain
  walk reads has the reference's type in Source/net_buf.h:394-598 (skipped where the reference tree
  is absent, e.g. on the GPU box);
* host/net_util_mi355x.c compiles -Wall -Wextra -Werror -pedantic in both modes — standalone and
  -DNETCSUM_IN_STACK against stack headers whose NET_BUF layout differs from the template mirror —
  with and without the NET_ERR_CFG_ARG_CHK_DBG_EN checks (tests/c/Makefile);
* a plain C caller (tests/c/dropin_caller.c) runs every variant under -fsanitize=address,undefined
  (and once under -fsanitize=thread: two threads racing for the CRC table's one-time build, then
  walking chains):
  chains of 0-1000 buffers walked and compared with its own concatenation, the error paths of
  net_util.c:168-179,1566-1577,1637-1672 through the drop-in, two threads at once; without a GPU
  every device call must fail with NET_UTIL_ERR_MI355X_DEV (no fallback);
* the offload-seam burst caller (tests/c/burst_caller.c) builds standalone and in-stack against
  stand-in headers configured with every NET_*_CFG_CHK_SUM_OFFLOAD_{RX,TX}_EN enabled, and refuses to
  build against a stack whose offload flags are off (the adapters replace the stack's checksum calls).
"""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/Source"
CDIR = os.path.join(REPO, "tests", "c")
VARIANTS = ["standalone_asan", "dbg_asan", "instack_asan", "instack_dbg_asan", "burst_asan", "burst_instack_asan", "tsan"]
FUNCS = ["NetUtil_16BitOnesCplChkSumHdrCalc", "NetUtil_16BitOnesCplChkSumHdrVerify",
         "NetUtil_16BitOnesCplChkSumDataCalc", "NetUtil_16BitOnesCplChkSumDataVerify",
         "NetUtil_32BitCRC_Calc", "NetUtil_32BitCRC_CalcCpl", "NetUtil_32BitReflect"]


def _prototype(text, name):
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    m = re.search(r"(\w+)\s+" + name + r"\s*\(([^)]*)\)\s*;", text)
    assert m, f"{name} not declared"
    return " ".join(f"{m.group(1)} {name} ( {m.group(2)} )".replace("*", " * ").replace(",", " , ").split())


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present (GPU box)")
def test_prototypes_match_reference_token_for_token():
    ref = open(os.path.join(REF, "net_util.h")).read()
    ours = open(os.path.join(REPO, "include", "netcsum_mi355x.h")).read()
    stand_in = open(os.path.join(REPO, "tests", "instack", "net_util.h")).read()
    for f in FUNCS:
        assert _prototype(ours, f) == _prototype(ref, f)
        assert _prototype(stand_in, f) == _prototype(ref, f)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present (GPU box)")
def test_netbuf_fields_have_reference_types():
    ref = open(os.path.join(REF, "net_buf.h")).read()
    fields = {"NextBufPtr": "NET_BUF *", "ProtocolHdrType": "NET_PROTOCOL_TYPE", "ICMP_MsgIx": "CPU_INT16U",
              "ICMP_HdrLen": "CPU_INT16U", "TransportHdrIx": "CPU_INT16U", "TransportHdrLen": "CPU_INT16U",
              "DataLen": "NET_BUF_SIZE", "TotLen": "NET_BUF_SIZE", "DataPtr": "CPU_INT08U *"}
    for hdr in (ref, open(os.path.join(REPO, "tests", "instack", "net_buf.h")).read()):
        for name, typ in fields.items():
            m = re.search(r"^\s*(\w+)\s*(\*?)\s*" + name + r"\s*;", hdr, flags=re.M)
            assert m, name
            assert (m.group(1) + (" *" if m.group(2) else "")) == typ, (name, m.group(0))
    assert re.search(r"typedef\s+CPU_INT16U\s+NET_BUF_SIZE\s*;", ref)


@pytest.fixture(scope="module")
def callers():
    r = subprocess.run(["make", "-s", "-C", CDIR], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return {v: os.path.join(CDIR, "build", v) for v in VARIANTS}


@pytest.mark.parametrize("variant", VARIANTS)
def test_c_caller_under_sanitizers(callers, variant):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    env.pop("NETCSUM_EXPECT_GPU", None)
    r = subprocess.run([callers[variant]], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert r.stdout.startswith("ok "), r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
    assert "ThreadSanitizer" not in r.stderr


def test_burst_caller_requires_the_offload_configuration():
    """In-stack, burst_caller.c compiles only when the stack maps its offload flags to the
    NET_*_CHK_SUM_OFFLOAD_* macros its call sites test (Source/net_cfg_net.h:174-190, 305-366)."""
    inc = ["-I" + os.path.join(REPO, "tests", "instack"), "-I" + os.path.join(REPO, "include")]
    src = os.path.join(CDIR, "burst_caller.c")
    on = subprocess.run(["gcc", "-std=c99", "-fsyntax-only", "-DNETCSUM_IN_STACK", "-DNETCSUM_TEST_OFFLOAD", *inc, src],
                        capture_output=True, text=True)
    assert on.returncode == 0, on.stderr
    off = subprocess.run(["gcc", "-std=c99", "-fsyntax-only", "-DNETCSUM_IN_STACK", *inc, src], capture_output=True, text=True)
    assert off.returncode != 0 and "OFFLOAD" in off.stderr
