"""Elastic data-dispatch master (reference: go/master/service_internal_test.go,
client_internal_test.go with InMemStore, client_test.go): tasks are handed out
once per pass, timed-out / failed tasks are re-dispatched, repeatedly failing tasks
are dropped, the state survives a master restart, one master per store."""
import threading
import time

import pytest

from paddle_amd.distributed import master as M
from paddle_amd.io.recordio import RecordIOWriter


def _dataset(tmp_path, files=3, per_file=10):
    paths = []
    for f in range(files):
        p = str(tmp_path / f"part-{f}.recordio")
        w = RecordIOWriter(p, max_num_records=4)
        for r in range(per_file):
            w.write(f"{f}:{r}".encode())
        w.close()
        paths.append(p)
    return str(tmp_path / "part-*.recordio"), {f"{f}:{r}".encode() for f in range(files) for r in range(per_file)}


def test_two_trainers_consume_a_pass_exactly_once(tmp_path):
    pat, want = _dataset(tmp_path)
    svc = M.MasterService(M.FileStore(str(tmp_path / "master.json")), chunks_per_task=1, timeout_s=30)
    srv = M.MasterServer(svc)
    c0 = M.MasterClient(srv.endpoint)
    c0.set_dataset([pat], 5)
    got = [[], []]

    def trainer(i):
        c = M.MasterClient(srv.endpoint)
        got[i] = list(c.records(0))
        c.close()

    ts = [threading.Thread(target=trainer, args=(i,)) for i in range(2)]
    [t.start() for t in ts]
    [t.join(30) for t in ts]
    allr = got[0] + got[1]
    assert sorted(allr) == sorted(want) and len(allr) == len(want)
    assert c0.status()["cur_pass"] == 1
    with pytest.raises(M.PassBefore):
        c0.get_task(0)
    c0.close()
    srv.stop()


def test_timeout_redispatch_and_failure_max(tmp_path):
    pat, want = _dataset(tmp_path, files=1, per_file=4)
    svc = M.MasterService(M.InMemStore(), chunks_per_task=1, timeout_s=0.2, failure_max=1)
    svc.set_dataset([pat], 2)                         # 2 tasks
    t = svc.get_task(0)                               # a trainer takes it ... and dies
    time.sleep(0.5)
    assert svc.status()["todo"] == 2                  # re-queued after the timeout
    # a stale report (old epoch) from the dead trainer is ignored
    t2 = [svc.get_task(0), svc.get_task(0)]
    assert svc.task_failed(t["id"], t["epoch"]) in (True, False)
    st = svc.status()
    assert st["pending"] + st["todo"] == 2
    # the timed-out task fails once more -> exceeds failure_max=1 -> dropped to failed
    bad = [x for x in t2 if x["id"] == t["id"]][0]
    svc.task_failed(bad["id"], bad["epoch"])
    assert svc.status()["failed"] == 1
    # the other task fails once -> re-queued and handed out again
    ok = [x for x in t2 if x["id"] != t["id"]][0]
    svc.task_failed(ok["id"], ok["epoch"])
    assert svc.get_task(0)["id"] == ok["id"]
    svc.shutdown()


def test_master_recovers_from_store_and_holds_leadership(tmp_path):
    pat, _ = _dataset(tmp_path, files=2, per_file=4)
    store_path = str(tmp_path / "m.json")
    svc = M.MasterService(M.FileStore(store_path), timeout_s=30)
    svc.set_dataset([pat], 4)
    t = svc.get_task(0)
    svc.task_finished(t["id"])
    before = svc.status()
    with pytest.raises(RuntimeError):                 # one leader per store
        st2 = M.FileStore(store_path)
        st2.acquire_leader = lambda timeout=0.2, s=st2: M.FileStore.acquire_leader(s, timeout)
        M.MasterService(st2)
    svc.shutdown()                                    # master dies; a new one recovers the state
    svc2 = M.MasterService(M.FileStore(store_path), timeout_s=30)
    assert svc2.status() == before
    ids = {svc2.get_task(0)["id"]}
    assert t["id"] not in ids
    svc2.shutdown()


def test_request_save_model_elects_one_trainer():
    svc = M.MasterService(M.InMemStore())
    assert svc.request_save_model("t0", 10.0) is True
    assert svc.request_save_model("t1", 10.0) is False
    assert svc.request_save_model("t0", 10.0) is True
    svc.shutdown()
