"""Config loader parity (reference cluster/config_test.go:9-45) + YAML subset."""
import json
import os

import pytest

from ptype_amd import _core
from ptype_amd import cluster as C

TD = os.path.join(os.path.dirname(__file__), "testdata")


def test_config_from_file_simple():
    cfg = C.ConfigFromFile(os.path.join(TD, "ping.yml"))
    assert cfg.member is not None  # etcdConfig loaded ("not our responsibility to test")
    assert (cfg.service_name, cfg.node_name, cfg.port, cfg.etcd_config_file, cfg.debug) == (
        "ping", "node1", 3000, "node1.yml", True)
    assert cfg.initial_cluster_client_urls == []
    m = cfg.member
    assert m.name == "node1" and m.dir == "tmp1"
    assert m.lpurls == ["http://127.0.0.1:12380"] and m.lcurls == ["http://127.0.0.1:12379"]
    assert m.initial_cluster == "node1=http://127.0.0.1:12380"
    assert m.cluster_state == "new" and m.initial_cluster_token == "etcd-cluster"
    assert m.strict_reconfig_check is False and m.logger == "zap"


def test_config_from_file_bad():
    # `service_name: 5` is a YAML number: it cannot decode into a string field
    with pytest.raises(C.ConfigError, match="cannot unmarshal number into Go struct field Config.service_name"):
        C.ConfigFromFile(os.path.join(TD, "bad_config.yml"))


def test_config_missing_files(tmp_path):
    with pytest.raises(C.ConfigError, match="failed to read cluster config"):
        C.ConfigFromFile(str(tmp_path / "nope.yml"))
    p = tmp_path / "a.yml"
    p.write_text("service_name: s\netcd_config_file: missing.yml\n")
    with pytest.raises(C.ConfigError, match="failed to read etcd config from missing.yml"):
        C.ConfigFromFile(str(p))


def test_config_member_validation(tmp_path):
    (tmp_path / "m.yml").write_text("name: x\nheartbeat-interval: 500\nelection-timeout: 1000\n")
    p = tmp_path / "a.yml"
    p.write_text("service_name: s\netcd_config_file: m.yml\n")
    with pytest.raises(C.ConfigError, match="should be at least as 5 times"):
        C.ConfigFromFile(str(p))
    (tmp_path / "m.yml").write_text("name: x\ninitial-cluster-state: weird\n")
    with pytest.raises(C.ConfigError, match="unexpected clusterState"):
        C.ConfigFromFile(str(p))
    (tmp_path / "m.yml").write_text("name: x\nlisten-client-urls: http://example.com:2379\n")
    with pytest.raises(C.ConfigError, match="expected IP in URL for binding"):
        C.ConfigFromFile(str(p))


def test_config_types_and_gpu_section(tmp_path):
    (tmp_path / "m.yml").write_text("name: x\n")
    p = tmp_path / "a.yml"
    p.write_text("service_name: 'calc'\nport: \"3000\"\netcd_config_file: m.yml\n")
    with pytest.raises(C.ConfigError, match="cannot unmarshal string into Go struct field Config.port of type int"):
        C.ConfigFromFile(str(p))
    p.write_text(
        "service_name: calc\nnode_name: node\nport: 31234\netcd_config_file: m.yml\n"
        "initial_cluster_client_urls:\n  - http://127.0.0.1:2379\n  - http://127.0.0.1:2479\n"
        "debug: yes\nunknown_key: ignored\n"
        "gpu:\n  device: 3\n  ring: 1024\n  actors: 4096\n  delay_us: 250000\n")
    cfg = C.ConfigFromFile(str(p))
    assert cfg.initial_cluster_client_urls == ["http://127.0.0.1:2379", "http://127.0.0.1:2479"]
    assert cfg.debug is True and cfg.has_gpu
    assert (cfg.gpu.device, cfg.gpu.ring, cfg.gpu.actors, cfg.gpu.delay_us) == (3, 1024, 4096, 250000)
    p.write_text("service_name: c\netcd_config_file: m.yml\ngpu:\n  ring: 1000\n")
    with pytest.raises(C.ConfigError, match="power of two"):
        C.ConfigFromFile(str(p))


def test_member_config_defaults_and_flow_seq(tmp_path):
    m = C.member_config()
    assert m.name == "default" and m.lpurls == ["http://localhost:2380"] and m.cluster_state == "new"
    assert m.effective_initial_cluster() == "default=http://localhost:2380"
    (tmp_path / "m.yml").write_text(
        "name: n3\nlisten-peer-urls: http://127.0.0.1:32380,http://127.0.0.1:32480\n"
        "initial-cluster: n1=http://127.0.0.1:1, n3=http://127.0.0.1:32380,n3=http://127.0.0.1:32480\n")
    mm = _core.MemberConfig.from_file(str(tmp_path / "m.yml"))
    assert mm.lpurls == ["http://127.0.0.1:32380", "http://127.0.0.1:32480"]
    assert mm.apurls == mm.lpurls  # advertise defaults to listen
    mm.validate()


@pytest.mark.parametrize(
    "text,expect",
    [
        ("a: 1\nb: two\nc: 'x # y'\nd: \"q\\\"\"\n", {"a": 1, "b": "two", "c": "x # y", "d": 'q"'}),
        ("list:\n  - 1\n  - b\nflow: [x, 'y', 2]\nm: {k: v, n: 3}\n", {"list": [1, "b"], "flow": ["x", "y", 2], "m": {"k": "v", "n": 3}}),
        ("outer:\n  inner:\n    leaf: true\n  other: ~\n", {"outer": {"inner": {"leaf": True}, "other": None}}),
        ("seq:\n- name: a\n  v: 1\n- name: b\n  v: 2\n", {"seq": [{"name": "a", "v": 1}, {"name": "b", "v": 2}]}),
        ("# comment only\nk: it's\n", {"k": "it's"}),
    ],
)
def test_yaml_subset(text, expect):
    assert json.loads(_core.yaml_to_json(text)) == expect


def test_yaml_errors():
    with pytest.raises(C.PtypeError):
        _core.yaml_to_json("a: 'unterminated\n")
    with pytest.raises(C.PtypeError, match="duplicate key"):
        _core.yaml_to_json("a: 1\na: 2\n")


def test_path_join_matches_go_filepath():
    assert _core.path_join("store", "hello") == "store/hello"
    assert _core.path_join("store", "a/../b/") == "store/b"
    assert _core.path_join("store", "") == "store"
    assert _core.etcd_key("services", "foo", "node1") == "services/foo/node1/"
    assert _core.etcd_key("services", "foo") == "services/foo/"
