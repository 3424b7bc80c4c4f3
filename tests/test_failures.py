"""Failure paths of group formation, bootstrap and the direct collectives (advisor
findings on direct.cpp): a failure on one rank must come back as an error on every rank, never as a
peer blocked in a barrier, and a rendezvous file an earlier job left behind must never be taken.

Every multi-rank case runs in a child process under a hard timeout, so a regression shows up as a
failed test, not a hung suite.  Fault injection: DCCL_FAULT_INJECT=<site>:<rank> (comm.hpp).
"""
import ctypes
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_child(code: str, env: dict, timeout: float = 60.0) -> dict:
    full = {**os.environ, **env, "PYTHONPATH": ROOT}
    p = subprocess.run([sys.executable, "-c", textwrap.dedent(code)], env=full, capture_output=True, text=True,
                       timeout=timeout)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


JOIN_CHILD = """
import ctypes, json, threading
import dccl_amd
W = int(__import__("os").environ["W"])
rcs, handles = [None] * W, [None] * W

def rank(r):
    h = ctypes.c_void_p()
    rcs[r] = dccl_amd.lib.dccl_comm_init_rank(ctypes.byref(h), W, r)
    handles[r] = h.value

ts = [threading.Thread(target=rank, args=(r,)) for r in range(W)]
[t.start() for t in ts]
[t.join(30) for t in ts]
hung = [r for r, t in enumerate(ts) if t.is_alive()]
print(json.dumps({"rcs": rcs, "hung": hung, "handles": [h is not None for h in handles]}))
"""


@pytest.mark.parametrize("W,bad", [(2, 1), (3, 0), (4, 2)])
def test_join_failure_reaches_every_rank_cpu(W, bad):
    """One rank fails after it was counted into the group (event creation): every rank returns an error
    (the failing one its own code, the others ncclRemoteError) and nobody waits forever."""
    res = run_child(JOIN_CHILD, {"W": str(W), "DCCL_FAULT_INJECT": f"join_events:{bad}"})
    assert res["hung"] == []
    assert res["rcs"][bad] == 1
    assert all(rc == 6 for r, rc in enumerate(res["rcs"]) if r != bad), res
    assert not any(res["handles"])


def test_join_without_fault_then_finalize_cpu():
    code = JOIN_CHILD + """
import dccl_amd as d
fin = [None] * W
def fin_rank(r):
    h = handles[r]
    fin[r] = d.lib.dccl_comm_finalize(ctypes.c_void_p(h)) if h else None
ts = [threading.Thread(target=fin_rank, args=(r,)) for r in range(W)]
[t.start() for t in ts]
[t.join(30) for t in ts]
print(json.dumps({"rcs": rcs, "fin": fin}))
"""
    res = run_child(code, {"W": "3", "DCCL_FAULT_INJECT": ""})
    assert res["rcs"] == [0, 0, 0] and res["fin"] == [0, 0, 0]


# ---------------------------------------------------------------------------------------------
# bootstrap rendezvous files (bootstrap.cpp)
# ---------------------------------------------------------------------------------------------
def _start_time(pid: int) -> int:
    line = open(f"/proc/{pid}/stat").read()
    return int(line[line.rindex(")") + 2:].split()[19])


def _stamp(pid: int, start: int, world: int, payload: bytes, gen: int = 1) -> str:
    return f"DCCLRDV2 {pid} {start} {gen} {world} {payload.hex()}\n"


@pytest.fixture()
def rdv(tmp_path, monkeypatch):
    monkeypatch.setenv("DCCL_BOOTSTRAP_DIR", str(tmp_path))
    monkeypatch.setenv("DCCL_BOOTSTRAP_TAG", "t_stale")
    monkeypatch.setenv("DCCL_BOOTSTRAP_TIMEOUT_S", "0.5")
    return tmp_path / "dccl_rccl_uid_t_stale"


def _read_id(world=2, rank=1):
    import dccl_amd
    buf = ctypes.create_string_buffer(128)
    rc = dccl_amd.lib.dccl_bootstrap_unique_id(rank, world, buf)
    return rc, buf.raw


def test_bootstrap_rejects_stale_file_cpu(rdv):
    """A file stamped by a process that is gone (an earlier job on the same tag) times out instead of
    handing a dead RCCL id to ncclCommInitRank."""
    child = subprocess.Popen(["true"])
    child.wait()
    dead_pid = child.pid
    uid = bytes(range(128))
    rdv.write_text(_stamp(dead_pid, 12345, 2, uid))
    rc, _ = _read_id()
    assert rc == 2
    # a round-1 style file (the raw 128-byte id, no stamp) is not taken either
    rdv.write_bytes(uid)
    assert _read_id()[0] == 2


def test_bootstrap_accepts_live_publisher_cpu(rdv):
    uid = bytes((7 * i + 3) % 256 for i in range(128))
    rdv.write_text(_stamp(os.getpid(), _start_time(os.getpid()), 2, uid))
    rc, got = _read_id()
    assert rc == 0 and got == uid
    # right publisher, wrong world size: another job's file
    rdv.write_text(_stamp(os.getpid(), _start_time(os.getpid()), 3, uid))
    assert _read_id()[0] == 2
    # the live pid but another start time: a recycled pid
    rdv.write_text(_stamp(os.getpid(), _start_time(os.getpid()) + 1, 2, uid))
    assert _read_id()[0] == 2


def test_bootstrap_two_groups_same_tag_cpu(rdv):
    """the same live rank 0 forms a second group under the same tag.  A peer that polls before rank 0
    republishes must not take the first group's id (it would join a finished RCCL bootstrap and hang); it
    waits for the new publication.  dccl_bootstrap_done then removes the file, as ncclCommInit does."""
    import dccl_amd
    first = ctypes.create_string_buffer(128)
    assert dccl_amd.lib.dccl_bootstrap_unique_id(0, 2, first) == 0  # rank 0 publishes group 1's id
    rc, got = _read_id()
    assert rc == 0 and got == first.raw
    # group 2: rank 1 polls before rank 0 republished -> times out instead of returning the old id
    assert _read_id()[0] == 2
    second = ctypes.create_string_buffer(128)
    assert dccl_amd.lib.dccl_bootstrap_unique_id(0, 2, second) == 0
    assert second.raw != first.raw
    rc, got = _read_id()
    assert rc == 0 and got == second.raw
    # every reader of the world took it: the file is gone, nobody can take it again
    assert not rdv.exists() and not list(rdv.parent.glob(rdv.name + ".took.*"))
    rc, got = _read_id(rank=1, world=2)
    assert rc == 2
    # with more readers the file stays until the last one took it; dccl_bootstrap_done on rank 0 removes it
    third = ctypes.create_string_buffer(128)
    assert dccl_amd.lib.dccl_bootstrap_unique_id(0, 3, third) == 0
    assert _read_id(world=3, rank=1) == (0, third.raw) and rdv.exists()
    assert dccl_amd.lib.dccl_bootstrap_done(1, 3) == 0 and rdv.exists()  # not rank 0: nothing removed
    assert dccl_amd.lib.dccl_bootstrap_done(0, 3) == 0 and not rdv.exists()
    assert _read_id()[0] == 2
    assert dccl_amd.lib.dccl_bootstrap_done(2, 2) == 4 and dccl_amd.lib.dccl_bootstrap_done(0, 0) == 4


_READER = r'''
import ctypes, json, os, sys
sys.path.insert(0, os.environ["ROOT"])
import dccl_amd
buf = ctypes.create_string_buffer(128)
rc = dccl_amd.lib.dccl_bootstrap_unique_id(1, 2, buf)
print(json.dumps({"rc": rc, "id": buf.raw.hex()}))
'''


def test_bootstrap_fresh_process_never_takes_old_id_cpu(rdv):
    """readers in separate processes.  Rank 0 publishes without ever calling dccl_bootstrap_done;
    once its group's readers took the id, a freshly started process polling the same tag must not get it
    (it would join a group that already formed); it gets the next publication."""
    import json as _json
    import dccl_amd
    env = {**os.environ, "ROOT": os.path.dirname(os.path.dirname(os.path.abspath(__file__)))}

    def reader():
        p = subprocess.run([sys.executable, "-c", _READER], env=env, capture_output=True, text=True, timeout=120)
        assert p.returncode == 0, p.stderr[-2000:]
        return _json.loads(p.stdout.strip().splitlines()[-1])

    first = ctypes.create_string_buffer(128)
    assert dccl_amd.lib.dccl_bootstrap_unique_id(0, 2, first) == 0
    got = reader()
    assert got["rc"] == 0 and bytes.fromhex(got["id"]) == first.raw
    assert reader()["rc"] == 2  # a new process: the old id is gone, it times out
    second = ctypes.create_string_buffer(128)
    assert dccl_amd.lib.dccl_bootstrap_unique_id(0, 2, second) == 0
    got = reader()
    assert got["rc"] == 0 and bytes.fromhex(got["id"]) == second.raw != first.raw


def test_bootstrap_argument_checks_cpu():
    import dccl_amd
    buf = ctypes.create_string_buffer(128)
    assert dccl_amd.lib.dccl_bootstrap_unique_id(2, 2, buf) == 4
    assert dccl_amd.lib.dccl_bootstrap_unique_id(0, 0, buf) == 4
    assert dccl_amd.lib.dccl_bootstrap_unique_id(0, 2, None) == 4


# ---------------------------------------------------------------------------------------------
# direct collectives: one rank's combine fails
# ---------------------------------------------------------------------------------------------
DIRECT_CHILD = """
import json, os, threading
import numpy as np
import dccl_amd
W, kind = int(os.environ["W"]), os.environ["KIND"]
n = 1024 * W
rcs, hung = [None] * W, []
def body(r):
    comm = dccl_amd.Comm.in_process(W, r)
    try:
        if kind == "device":
            import torch
            x = torch.full((n,), float(r + 1), device="cuda")
            st = torch.cuda.current_stream().cuda_stream
            rcs[r] = [comm.all_reduce(x.data_ptr(), x.data_ptr(), n, 7, 0, st),
                      comm.reduce_scatter(x.data_ptr(), x.data_ptr(), n // W, 7, 0, st)]
        else:
            x = np.full(n, r + 1, np.float32)
            y = np.zeros(n // W, np.float32)
            rcs[r] = [comm.all_reduce(x.ctypes.data, x.ctypes.data, n, 7, 0),
                      comm.reduce_scatter(x.ctypes.data, y.ctypes.data, n // W, 7, 0)]
    finally:
        comm.finalize()
ts = [threading.Thread(target=body, args=(r,)) for r in range(W)]
[t.start() for t in ts]
[t.join(60) for t in ts]
print(json.dumps({"rcs": rcs, "hung": [r for r, t in enumerate(ts) if t.is_alive()]}))
"""


@pytest.mark.parametrize("W,bad", [(2, 1), (3, 0)])
def test_direct_host_combine_failure_no_hang_cpu(W, bad):
    """Host buffers take the direct choreography; without a GPU every rank's staged combine fails, and with
    the injected fault one rank fails first: no rank may wait forever, every rank reports an error."""
    res = run_child(DIRECT_CHILD, {"W": str(W), "KIND": "host", "DCCL_FAULT_INJECT": f"direct_combine:{bad}"})
    assert res["hung"] == []
    for r in range(W):
        assert all(rc != 0 for rc in res["rcs"][r]), res


@pytest.mark.gpu
@pytest.mark.parametrize("W,bad", [(2, 1), (3, 0), (4, 3)])
@pytest.mark.parametrize("kind", ["device", "host"])
def test_direct_combine_failure_reaches_every_rank(gpu, W, bad, kind):
    """On the GPU only the injected rank fails: it returns its own code (1), every peer ncclRemoteError (6),
    for all_reduce (three phase points) and reduce_scatter alike."""
    res = run_child(DIRECT_CHILD, {"W": str(W), "KIND": kind, "DCCL_FAULT_INJECT": f"direct_combine:{bad}"},
                    timeout=120)
    assert res["hung"] == []
    for r in range(W):
        want = 1 if r == bad else 6
        assert res["rcs"][r] == [want, want], res


# ---------------------------------------------------------------------------------------------
# the IPC transport after a failure: sticky abort, finalize still releases everything
# ---------------------------------------------------------------------------------------------
IPC_FAIL_CHILD = """
import glob, json, os
import torch
import dccl_amd
import time
W, r = int(os.environ["W"]), int(os.environ["RANK_ID"])
torch.cuda.set_device(0)
if r == int(os.environ.get("LATE_RANK", "-1")):  # joins late: its peers wait at the join barrier meanwhile
    time.sleep(float(os.environ["LATE_S"]))
comm = dccl_amd.Comm.ipc(W, r)
n = 1024 * W
x = torch.full((n,), float(r + 1), device="cuda")
st = torch.cuda.current_stream().cuda_stream
first = comm.all_reduce(x.data_ptr(), x.data_ptr(), n, 7, 0, st)
torch.cuda.synchronize()
second = comm.all_reduce(x.data_ptr(), x.data_ptr(), n, 7, 0, st)   # the abort is sticky on this transport
torch.cuda.synchronize()
fin = comm.finalize()
print(json.dumps({"first": first, "second": second, "finalize": fin, "pid": os.getpid()}))
"""


@pytest.mark.gpu
def test_ipc_failure_is_sticky_and_finalize_releases(gpu, tmp_path):
    """On the IPC transport one rank's failed combine aborts the group: every rank gets an error, the next
    collective returns ncclRemoteError at once (include/dccl/dccl_comm.h), and finalize still returns,
    unmaps the shared segment and leaves no /dev/shm segment or rendezvous file behind."""
    import uuid
    W, tag = 2, "ipcfail_" + uuid.uuid4().hex[:10]
    env = {**os.environ, "PYTHONPATH": ROOT, "W": str(W), "DCCL_BOOTSTRAP_TAG": tag, "DCCL_BOOTSTRAP_DIR": str(tmp_path),
           "DCCL_FAULT_INJECT": "direct_combine:1", "DCCL_IPC_TIMEOUT_S": "20"}
    ps = [subprocess.Popen([sys.executable, "-c", textwrap.dedent(IPC_FAIL_CHILD)], env={**env, "RANK_ID": str(r)},
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(W)]
    outs = []
    try:
        for p in ps:
            o, e = p.communicate(timeout=120)
            assert p.returncode == 0, e[-2000:]
            outs.append(json.loads(o.strip().splitlines()[-1]))
    finally:
        for p in ps:
            if p.poll() is None:
                p.kill()
                p.wait()
    assert outs[1]["first"] == 1 and outs[0]["first"] == 6, outs
    assert outs[0]["second"] == 6 and outs[1]["second"] != 0, outs
    assert all(o["finalize"] in (0, 6) for o in outs), outs
    import glob
    assert not glob.glob(f"/dev/shm/dccl_ipc_{outs[0]['pid']}_*"), "rank 0's segment left behind"
    assert not list(tmp_path.iterdir()), list(tmp_path.iterdir())


# ---------------------------------------------------------------------------------------------
# a peer whose process this rank cannot see (another pid namespace, /proc hidepid)
# ---------------------------------------------------------------------------------------------
IPC_HIDDEN_CHILD = """
import json, os
import torch
import dccl_amd
import time
W, r = int(os.environ["W"]), int(os.environ["RANK_ID"])
torch.cuda.set_device(0)
if r == int(os.environ.get("LATE_RANK", "-1")):  # joins late: its peers wait at the join barrier meanwhile
    time.sleep(float(os.environ["LATE_S"]))
comm = dccl_amd.Comm.ipc(W, r)
n = 1024 * W
x = torch.full((n,), float(r + 1), device="cuda")
st = torch.cuda.current_stream().cuda_stream
rcs = []
for _ in range(3):
    x.fill_(float(r + 1))
    torch.cuda.synchronize()
    rcs.append(comm.all_reduce(x.data_ptr(), x.data_ptr(), n, 7, 0, st))
    torch.cuda.synchronize()
ok = bool(torch.all(x == float(W * (W + 1) // 2)))
print(json.dumps({"rcs": rcs, "ok": ok, "finalize": comm.finalize()}))
"""


@pytest.mark.gpu
@pytest.mark.parametrize("W,late", [(2, None), (3, 2), (4, 0)])
def test_ipc_invisible_peer_turns_liveness_off(gpu, tmp_path, W, late):
    """A rank whose peers cannot see its process (DCCL_FAULT_INJECT=hidden_pid:1 publishes a pid that does not
    exist) must not be taken for dead: its peers turn the liveness check off for that communicator at join and
    say so once on stderr, and every collective succeeds (before, any barrier wait over 100 ms became
    ncclRemoteError).  With a rank joining 700 ms late, the others wait at the join barrier after the hidden
    rank has published its pid: that wait runs without the liveness check, or it would take the
    hidden rank for dead and abort every rank's init."""
    import uuid
    tag = "ipchide_" + uuid.uuid4().hex[:10]
    env = {**os.environ, "PYTHONPATH": ROOT, "W": str(W), "DCCL_BOOTSTRAP_TAG": tag, "DCCL_BOOTSTRAP_DIR": str(tmp_path),
           "DCCL_FAULT_INJECT": "hidden_pid:1"}
    if late is not None:
        env.update(LATE_RANK=str(late), LATE_S="0.7")
    env.pop("DCCL_IPC_TIMEOUT_S", None)
    ps = [subprocess.Popen([sys.executable, "-c", textwrap.dedent(IPC_HIDDEN_CHILD)], env={**env, "RANK_ID": str(r)},
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(W)]
    outs, errs = [], []
    try:
        for p in ps:
            o, e = p.communicate(timeout=120)
            assert p.returncode == 0, e[-2000:]
            outs.append(json.loads(o.strip().splitlines()[-1]))
            errs.append(e)
    finally:
        for p in ps:
            if p.poll() is None:
                p.kill()
                p.wait()
    assert all(o["rcs"] == [0, 0, 0] and o["ok"] and o["finalize"] == 0 for o in outs), outs
    for p in range(W):  # every rank but the hidden one sees an invisible peer; the hidden rank sees everyone
        if p == 1:
            assert "liveness check off" not in errs[p], errs[p][-2000:]
        else:
            assert "liveness check off for this communicator" in errs[p], (p, errs[p][-2000:])
