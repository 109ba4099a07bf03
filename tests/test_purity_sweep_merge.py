"""CPU test of the C5 (BASELINE configs[4]) sweep's multi-rank path: scripts/purity_sweep.py
under torch.distributed.run with 2 gloo ranks and a stubbed scorer (--stub).  Every rank
writes its round-robin share of the vectors to its rank file and rank 0 merges them after
a barrier: the merged records cover every vector of the sweep exactly once and the summary
counts them."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_rank_sweep_merge(tmp_path):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = tmp_path / "purity"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29641",
           os.path.join(REPO, "scripts", "purity_sweep.py"), "--stub", "--npoints", "20",
           "--out-dir", str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    recs = [d for d in lines if not d.get("summary")]
    summ = [d for d in lines if d.get("summary")]
    assert len(summ) == 1 and summ[0]["gpus"] == 2
    # the full vector list of the sweep, each exactly once, dealt round-robin
    sys.path[:0] = [os.path.join(REPO, "ska-pst-dsp-model_amd")]
    from ska_pst_dsp_model_amd import verify
    al = verify.performance_alignment(4096, "8/7", 512, 128, 100353, 3, 0, 0)
    items = verify.sweep_vectors(al, 20, 3) + [("comb", 32), ("square_wave", 3981)]
    got = sorted((d["domain"], d["param"]) for d in recs)
    assert got == sorted(items)
    assert {d["rank"] for d in recs} == {0, 1}
    for rank in (0, 1):
        mine = sorted((d["domain"], d["param"]) for d in recs if d["rank"] == rank)
        assert mine == sorted(items[rank::2])  # round-robin (verify.shard)
    s = summ[0]
    assert s["vectors"] == len(items) and s["tones"] == sum(k == "freq" for k, _ in items)
    assert s["impulses_at_expected_index"] == s["impulses_in_output"]
    assert sorted(os.listdir(out)) == ["rank0.jsonl", "rank1.jsonl"]
