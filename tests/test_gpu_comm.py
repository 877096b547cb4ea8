"""GPU tests of the multi-GPU exchange behind the C-ABI (osk_comm.hip): RCCL loaded and driven by
libosknn itself, no torch collective in the path.

The one-GPU box can only form world-1 communicators (RCCL refuses two ranks on one GPU), so these
tests check every entry point at world 1 — the id, both init flavours, the raw all-gather, the
padded shards-per-rank layout, the device and host search+merge entries — against the single-view
search and the oracle's coordinator merge.  The multi-rank logic of the same exchange (gathered
image layout, shardIndex of pad slots, the reduce) is covered on CPU with gloo world 2/3
(tests/test_distributed_cpu.py) and by the N = 2/4/8 rehearsal on one GPU (tools/gpu_rehearse.sh).
Reference semantics: S/action/search/SearchPhaseController.java:224-253 (mergeTopDocs, setShardIndex),
AbstractSearchAsyncAction.java:262-268 (one request per shard, loop index = shardIndex).
"""
import numpy as np
import pytest
import torch

from opensearch_amd import _lib, distributed as D, lucene as LU
from oracle import oracle as O

pytestmark = pytest.mark.gpu

COS = LU.VectorSimilarityFunction.COSINE


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def shardset():
    sizes = [9000, 4000, 12000]
    segs = [O.synth(0, n, 768, 60 + i, 3) for i, n in enumerate(sizes)]
    readers = [LU.GpuFlatVectorsReader("v", r, COS) for r in segs]
    si = [5, 2, 7]
    ds = LU.DeviceShardSet([[LU.LeafReaderContext(0, 0, r)] for r in readers], si)
    yield ds, segs, si
    ds.close()
    for r in readers:
        r.close()


def oracle(segs, si, q, k, from_, size, accept=None):
    lists = []
    for j, rows in enumerate(segs):
        ab = None if accept is None or accept[j] is None else O.bits_from_bool(accept[j])
        sc, dc, _ = O.exact_search(rows, q, k, int(COS), accept_bits=ab)
        lists.append((sc[: from_ + size], dc[: from_ + size]))
    return O.topdocs_merge(lists, from_, size, si)


def test_world1_rank_comm_info_and_raw_all_gather():
    comm = D.DeviceComm.init_rank(0, 0, 1, D.DeviceComm.unique_id())
    try:
        assert (comm.rank, comm.world, comm.n_local) == (0, 1, 1)
        src = torch.arange(1000, dtype=torch.int64, device="cuda")
        dst = torch.zeros_like(src)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            comm.all_gather(src, dst, s.cuda_stream)
        s.synchronize()
        assert torch.equal(src, dst)
    finally:
        comm.close()


@pytest.mark.parametrize("nq,k,from_,size,spr", [(1, 10, 0, 10, 3), (3, 10, 2, 8, 3), (5, 12, 0, 12, 5),
                                                  (2, 30, 10, 20, 4), (40, 10, 0, 10, 3)])
def test_shards_search_merge_device_world1(shardset, nq, k, from_, size, spr):
    """spr > the view's 3 shards exercises the padded layout (pad slots = empty lists)."""
    ds, segs, si = shardset
    comm = D.DeviceComm.init_rank(0, 0, 1, D.DeviceComm.unique_id())
    try:
        queries = O.synth(0, nq, 768, 70 + nq, 3)
        step = D.ShardSearchMerge(comm, ds.handle, spr, nq, k, from_, size, device=0)
        s = torch.cuda.Stream()
        dq = torch.from_numpy(queries).cuda()
        torch.cuda.synchronize()
        res = step(dq.data_ptr(), s.cuda_stream)
        s.synchronize()
        out = [t.cpu().numpy() for t in res]
        want = ds.search(queries, k, from_, size)
        for w, g in zip(want, out):
            if w.dtype == np.float32:
                assert np.array_equal(bits(w), bits(g))
            else:
                assert np.array_equal(w, g)
        for i in range(nq):
            es, ed, esh, et, em = oracle(segs, si, queries[i], k, from_, size)
            n = out[3][i]
            assert n == len(ed) and np.array_equal(out[1][i, :n], ed) and np.array_equal(out[2][i, :n], esh)
            assert np.array_equal(bits(out[0][i, :n]), bits(es)) and out[4][i] == et
    finally:
        comm.close()


def test_shards_search_merge_host_init_all_with_filters(shardset):
    ds, segs, si = shardset
    comm = D.DeviceComm.init_all([0])
    try:
        assert (comm.rank, comm.world, comm.n_local) == (0, 1, 1)
        rng = np.random.default_rng(3)
        queries = O.synth(0, 4, 768, 80, 3)
        for accept in (None, [rng.random(9000) < 0.02, None, rng.random(12000) < 0.3]):
            out = D.shards_search_merge(comm, [ds], queries, 10, 0, 10, accept)
            want = ds.search(queries, 10, 0, 10, accept=accept)
            for w, g in zip(want, out):
                assert np.array_equal(w.view(np.uint32) if w.dtype == np.float32 else w,
                                      g.view(np.uint32) if g.dtype == np.float32 else g)
            for i in range(len(queries)):
                es, ed, esh, _, _ = oracle(segs, si, queries[i], 10, 0, 10, accept)
                assert np.array_equal(out[1][i, : out[3][i]], ed) and np.array_equal(out[2][i, : out[3][i]], esh)
    finally:
        comm.close()


def test_comm_errors_are_codes(shardset):
    ds, _, _ = shardset
    comm = D.DeviceComm.init_rank(0, 0, 1, D.DeviceComm.unique_id())
    try:
        step = D.ShardSearchMerge(comm, ds.handle, 2, 1, 10, 0, 10, device=0)   # 3 shards > spr 2
        dq = torch.zeros((1, 768), dtype=torch.float32, device="cuda")
        with pytest.raises(_lib.OskError):
            step(dq.data_ptr(), torch.cuda.Stream().cuda_stream)
        with pytest.raises(_lib.OskError):
            D.DeviceComm.init_all([0, 0])
    finally:
        comm.close()


def test_queries_in_flight_on_views_and_streams(shardset):
    """bench.py's serving mode: F search threads, each with its own view over the same segments and its
    own stream, issue single-query steps round-robin through osk_shards_search_merge_device, so
    consecutive queries overlap on the device.  Every step must equal the serial search."""
    ds, segs, si = shardset
    leaves = ds.leaves
    extra = [LU.DeviceShardSet([[lf] for lf in leaves], si) for _ in range(2)]
    handles = [ds.handle] + [e.handle for e in extra]
    comm = D.DeviceComm.init_rank(0, 0, 1, D.DeviceComm.unique_id())
    try:
        F, n = len(handles), 24
        queries = O.synth(0, n, 768, 91, 3)
        dq = torch.from_numpy(queries).cuda()
        streams = [torch.cuda.Stream() for _ in range(F)]
        steps = [D.ShardSearchMerge(comm, h, 3, 1, 10, 0, 10, device=0) for h in handles]
        torch.cuda.synchronize()
        got = []
        for i in range(n):
            j = i % F
            res = steps[j](dq[i:i + 1].data_ptr(), streams[j].cuda_stream)
            with torch.cuda.stream(streams[j]):   # snapshot on the producing stream before slot j is reused
                got.append([t.clone() for t in res])
        torch.cuda.synchronize()
        want = ds.search(queries, 10, 0, 10)
        for i in range(n):
            g = [t.cpu().numpy()[0] for t in got[i]]
            assert np.array_equal(bits(g[0]), bits(want[0][i])) and np.array_equal(g[1], want[1][i])
            assert np.array_equal(g[2], want[2][i]) and g[3] == want[3][i] and g[4] == want[4][i]
    finally:
        comm.close()
        for e in extra:
            e.close()


def test_raw_all_gather_from_two_streams_keeps_call_order():
    """Collectives issued from different caller streams run in call order on the communicator's own
    exchange stream, each after the work its caller stream had enqueued."""
    comm = D.DeviceComm.init_rank(0, 0, 1, D.DeviceComm.unique_id())
    try:
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        a = torch.zeros(1 << 20, dtype=torch.int64, device="cuda")
        b = torch.empty_like(a)
        c = torch.empty_like(a)
        torch.cuda.synchronize()
        with torch.cuda.stream(s1):
            a.fill_(7)                       # enqueued on s1 before its gather
            comm.all_gather(a, b, s1.cuda_stream)
        with torch.cuda.stream(s2):
            s2.wait_stream(s1)
            comm.all_gather(b, c, s2.cuda_stream)
            d = c.sum()
        torch.cuda.synchronize()
        assert int(d) == 7 * (1 << 20) and torch.equal(b, a)
    finally:
        comm.close()
