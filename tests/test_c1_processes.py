"""BASELINE config C1 as the reference runs it: `dccl_cli -a all_reduce -t float32|uint32 -c 1024` with FOUR
PROCESSES over loopback (/root/reference/README.md:74-101; src/application/cli.cpp:360-381 one process per
rank, :380 sendbuf = memset(rank), :421-424 ncclAllReduce in place on sendbuf, host buffers).

Each rank is its own process.  The transport is test glue, not a product transport: a point-to-point
exchange over loopback TCP sockets (the stand-in for Derecho's OOB send / recv over its tcp provider,
internal_common.hpp:698-792), plugged in through dccl_comm_init_p2p (include/dccl/dccl_comm.h) with host
memory only.  The ring reduce-scatter + all-gather of this build run on it with the gfx950 combine for every
received chunk (host operands staged through the GPU), and every rank must end with the survey's known
answers (tests/golden/c1_ring.json): fp32 0x032b9394 after one all_reduce ... 0x7f800000
after 1000; uint32 0x06060606 ... 0x00000000.
"""
import json
import os
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RANK_CHILD = r"""
import ctypes, json, os, socket, struct, sys, threading, time
sys.path.insert(0, os.environ["ROOT"])
import numpy as np
import dccl_amd
W, rank, d = int(os.environ["W"]), int(os.environ["RANK"]), os.environ["RDV"]

# loopback TCP: one listening socket per rank, its port published in the rendezvous directory
ls = socket.socket()
ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
ls.bind(("127.0.0.1", 0))
ls.listen(W)
tmp = os.path.join(d, f"port{rank}.tmp")
open(tmp, "w").write(str(ls.getsockname()[1]))
os.rename(tmp, os.path.join(d, f"port{rank}"))

def port_of(p):
    path = os.path.join(d, f"port{p}")
    for _ in range(6000):
        if os.path.exists(path):
            return int(open(path).read())
        time.sleep(0.01)
    raise SystemExit(f"rank {p} never published its port")

out_sock, in_sock = {}, {}
def accept_all():
    for _ in range(W - 1):
        c, _ = ls.accept()
        c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        in_sock[struct.unpack("<I", c.recv(4, socket.MSG_WAITALL))[0]] = c
acc = threading.Thread(target=accept_all)
acc.start()
for p in range(W):
    if p != rank:
        s = socket.create_connection(("127.0.0.1", port_of(p)))
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        s.sendall(struct.pack("<I", rank))
        out_sock[p] = s
acc.join(60)

def recv_exact(s, n):
    buf = bytearray(n)
    view, got = memoryview(buf), 0
    while got < n:
        k = s.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("peer closed")
        got += k
    return bytes(buf)

def exchange(ctx, sbuf, sn, to, rbuf, rn, frm, stream):
    try:
        th = None
        if sbuf:  # send on a helper thread, so two ranks sending to each other never block each other
            data = struct.pack("<Q", sn) + ctypes.string_at(sbuf, sn)
            th = threading.Thread(target=out_sock[to].sendall, args=(data,))
            th.start()
        if rbuf:
            n = struct.unpack("<Q", recv_exact(in_sock[frm], 8))[0]
            if n != rn:
                return 5
            ctypes.memmove(rbuf, recv_exact(in_sock[frm], n), n)
        if th is not None:
            th.join()
        return 0
    except Exception:
        return 2  # ncclSystemError from the transport

fn = dccl_amd.P2P_EXCHANGE_FN(exchange)
h = ctypes.c_void_p()
rc = dccl_amd.lib.dccl_comm_init_p2p(ctypes.byref(h), W, rank, fn, None, 1)  # host buffers
assert rc == 0, rc
count, res = 1024, {}
if os.environ.get("MODE") == "all_gather":  # the transport alone (no combine): runs without a GPU
    mine = np.full(count, rank + 1, np.uint32)
    allv = np.zeros(count * W, np.uint32)
    for _ in range(20):
        rc = dccl_amd.lib.dccl_all_gather(mine.ctypes.data, allv.ctypes.data, count, 3, h, None)
        assert rc == 0, rc
    res["all_gather"] = [int(x) for x in allv[::count]]
    assert dccl_amd.lib.dccl_comm_finalize(h) == 0
    print(json.dumps({"rank": rank, "results": res}), flush=True)
    sys.exit(0)
for name, dt, npd in (("float32", 7, np.float32), ("uint32", 3, np.uint32)):
    buf = np.empty(count, npd)
    buf.view(np.uint8)[:] = rank  # memset(sendbuf, my_rank, ...), cli.cpp:380
    done, got = 0, {}
    for upto in (1, 2, 10, 1000):
        while done < upto:
            rc = dccl_amd.lib.dccl_all_reduce(buf.ctypes.data, buf.ctypes.data, count, dt, 0, h, None)
            assert rc == 0, (name, done, rc)
            done += 1
        u = np.unique(buf.view(np.uint32))
        got[str(upto)] = [f"0x{int(x):08x}" for x in u]
    res[name] = got
assert dccl_amd.lib.dccl_comm_finalize(h) == 0
print(json.dumps({"rank": rank, "results": res}), flush=True)
"""


def run_ranks(W, mode=""):
    with tempfile.TemporaryDirectory(prefix="dccl_c1_") as d:
        env = {**os.environ, "ROOT": ROOT, "W": str(W), "RDV": d, "MODE": mode}
        procs = [subprocess.Popen([sys.executable, "-c", RANK_CHILD], env={**env, "RANK": str(r)},
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(W)]
        outs = []
        try:
            for p in procs:
                o, e = p.communicate(timeout=240)
                outs.append((p.returncode, o, e))
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
                    p.wait()
    res = []
    for r, (rc, o, e) in enumerate(outs):
        assert rc == 0, f"rank {r}: {e[-2000:]}"
        res.append(json.loads(o.strip().splitlines()[-1])["results"])
    return res


def test_c1_transport_four_processes_cpu():
    """The 4-process loopback transport itself, through the ring all-gather (no combine, so no GPU)."""
    for res in run_ranks(4, "all_gather"):
        assert res["all_gather"] == [1, 2, 3, 4]


@pytest.mark.gpu
def test_c1_known_answers_four_processes(gpu):
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "c1_ring.json")))
    for r, res in enumerate(run_ranks(gold["world_size"])):
        for name in ("float32", "uint32"):
            for upto, want in gold[name].items():
                assert res[name][upto] == [want], (r, name, upto, res[name][upto], want)
