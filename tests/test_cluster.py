"""Cluster facade parity (reference cluster/cluster_test.go, ClusterSuite):
Join from ping.yml, then grow a cluster 1 -> 2 (learner add + promote) -> 3 (a
member with two peer/client URLs) -> close one -> 4.  Several control-plane
members run in one process on loopback ports, each with its own data dir, as
the reference runs several embedded etcd members in one test process."""
import os
import shutil

import pytest

from ptype_amd import _core
from ptype_amd import cluster as C

TD = os.path.join(os.path.dirname(__file__), "testdata")


@pytest.fixture
def workdir(tmp_path, monkeypatch):
    for f in ("ping.yml", "node1.yml"):
        shutil.copy(os.path.join(TD, f), tmp_path / f)
    monkeypatch.chdir(tmp_path)  # data-dir tmp1 is relative, like the reference
    monkeypatch.setenv("PTYPE_ADVERTISE_ADDR", "127.0.0.1")
    return tmp_path


def _ping_cfg(workdir, ports):
    cfg = C.ConfigFromFile(str(workdir / "ping.yml"))
    m = cfg.member
    pc, pp = ports(), ports()  # ping.yml pins 12379/12380; use free ports
    m.lcurls = [f"http://127.0.0.1:{pc}"]
    m.acurls = list(m.lcurls)
    m.lpurls = [f"http://127.0.0.1:{pp}"]
    m.apurls = list(m.lpurls)
    m.initial_cluster = f"node1=http://127.0.0.1:{pp}"
    m.heartbeat_ms, m.election_ms, m.unsafe_no_fsync = 50, 500, True
    cfg.member = m
    return cfg


def test_join(workdir, ports):
    cfg = _ping_cfg(workdir, ports)
    ctx = C.Context.with_cancel(None)
    c = C.Join(ctx, cfg)
    try:
        services = c.Registry.Services(ctx)
        assert services["ping"] == [C.Node("127.0.0.1", 3000)]
        assert os.path.isdir(workdir / "tmp1" / "member")  # WAL + snapshot live in data-dir
    finally:
        ctx.cancel()
        c.Close()


def _member_cfg(name, service, port, seed_url, n_urls, ports, workdir):
    peer = [f"http://127.0.0.1:{ports()}" for _ in range(n_urls)]
    client = [f"http://127.0.0.1:{ports()}" for _ in range(n_urls)]
    cfg = C.Config()
    cfg.service_name, cfg.node_name, cfg.port = service, name, port
    cfg.initial_cluster_client_urls = [seed_url]
    cfg.member = C.member_config(name=name, dir=str(workdir / f"tmp{name[-1]}"), lpurls=peer, lcurls=client,
                                 apurls=peer, acurls=client, cluster_state="existing", heartbeat_ms=50,
                                 election_ms=500, unsafe_no_fsync=True)
    return cfg


def test_member_add(workdir, ports):
    cfg = _ping_cfg(workdir, ports)
    ctx = C.Context.with_cancel(None)
    c = C.Join(ctx, cfg)
    opened = [c]
    try:
        assert len(c.MemberList(ctx)) == 1
        seed = cfg.member.lcurls[0]

        c2 = C.Join(ctx, _member_cfg("node2", "testservice", 3030, seed, 1, ports, workdir))
        opened.append(c2)
        members = c.MemberList(ctx)
        assert len(members) == 2 and not any(m.is_learner for m in members)  # promoted

        c3 = C.Join(ctx, _member_cfg("node3", "testservice2", 8080, seed, 2, ports, workdir))
        opened.append(c3)
        members = c.MemberList(ctx)
        assert len(members) == 3
        m3 = [m for m in members if m.name == "node3"][0]
        assert len(m3.peer_urls) == 2 and len(m3.client_urls) == 2

        # add a node with one faulty node in a three node cluster
        c3.Close()
        c4 = C.Join(ctx, _member_cfg("node4", "testservice3", 4040, seed, 1, ports, workdir))
        opened.append(c4)
        members = c.MemberList(ctx)
        assert len(members) == 4  # no MemberRemove: the closed member stays listed
        # every live member serves the replicated registry
        svcs = c4.Registry.Services(ctx)
        assert {"ping", "testservice", "testservice3"} <= set(svcs)
    finally:
        ctx.cancel()
        for x in reversed(opened):
            x.Close()


def test_join_existing_requires_seed_urls(workdir, ports):
    cfg = _member_cfg("node2", "s", 1, "http://127.0.0.1:1", 1, ports, workdir)
    cfg.initial_cluster_client_urls = []
    with pytest.raises(C.ConfigError, match="requires at least one client url"):
        C.Join(C.background(), cfg)


def test_initial_cluster_string_for_joiner(workdir, ports):
    """memberAdd (cluster.go:120-147): sorted name=url for self (every peer URL)
    plus every started member; an unstarted learner (empty name) is excluded."""
    cfg = _ping_cfg(workdir, ports)
    ctx = C.Context.with_cancel(None)
    c = C.Join(ctx, cfg)
    try:
        j = _member_cfg("node9", "s", 1, cfg.member.lcurls[0], 2, ports, workdir)
        s = _core.Cluster.join_existing_cluster(ctx, j)
        parts = s.split(",")
        assert parts == sorted(parts)
        assert f"node1={cfg.member.lpurls[0]}" in parts
        assert sum(p.startswith("node9=") for p in parts) == 2
        # node9 was added as a learner but never started: it is listed without a name
        names = [m.name for m in c.MemberList(ctx)]
        assert "" in names
        # a second joiner's initial-cluster excludes that unstarted member
        j2 = _member_cfg("node8", "s", 1, cfg.member.lcurls[0], 1, ports, workdir)
        parts2 = _core.Cluster.join_existing_cluster(ctx, j2).split(",")
        assert not any(p.startswith("node9=") for p in parts2)
        assert f"node1={cfg.member.lpurls[0]}" in parts2
        # re-adding the same peer URLs is refused
        with pytest.raises(C.PtypeError, match="Peer URLs already exists"):
            _core.Cluster.join_existing_cluster(ctx, j2)
    finally:
        ctx.cancel()
        c.Close()


def test_restart_recovers_state_from_wal(workdir, ports):
    cfg = _ping_cfg(workdir, ports)
    ctx = C.Context.with_cancel(None)
    c = C.Join(ctx, cfg)
    c.Store.Put(ctx, "persist", "me")
    mid = c.member_id
    c.Close()
    ctx.cancel()
    ctx2 = C.Context.with_cancel(None)
    c2 = C.Join(ctx2, cfg)  # same data dir: resumes log, membership and KV state
    try:
        assert c2.member_id == mid
        assert c2.Store.Get(ctx2, "persist") == ["me"]
        assert len(c2.MemberList(ctx2)) == 1
    finally:
        ctx2.cancel()
        c2.Close()
