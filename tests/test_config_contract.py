"""Configuration contracts (what the reference pins in tests/unittests/core/io/test_resolve_config.py
and test_config.py): config-file fetching, default options, environment variables, run metadata
with the user script and its git state, recursive right-most-wins merging, and the typed option
tree with value > env var > yaml > default precedence.  Written against this package's API."""
import os
import stat
import subprocess

import pytest

from metaopt_amd.core.config import Configuration, ConfigurationError
from metaopt_amd.io import resolve_config as rc


# ------------------------------------------------------------------ fetch_*
def test_fetch_config_no_hit():
    assert rc.fetch_config({"config": None}) == {} and rc.fetch_config({}) == {}


def test_fetch_config_from_path_and_file(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text("name: exp\nmax_trials: 5\nalgorithms:\n  asha:\n    seed: 1\n")
    want = {"name": "exp", "max_trials": 5, "algorithms": {"asha": {"seed": 1}}}
    assert rc.fetch_config({"config": str(p)}) == want
    with open(p) as f:
        f.read()                              # an already-consumed handle is rewound
        assert rc.fetch_config({"config": f}) == want


def test_fetch_config_empty_file(tmp_path):
    p = tmp_path / "e.yaml"
    p.write_text("")
    assert rc.fetch_config({"config": str(p)}) == {}


def test_fetch_default_options():
    d = rc.fetch_default_options()
    assert d["max_trials"] == float("inf") and d["worker_trials"] == float("inf")
    assert d["pool_size"] == 1 and d["algorithms"] == "random" and d["name"] is None
    assert set(d["database"]) == {"name", "type", "host", "port"}
    assert d["user"]


def test_fetch_env_vars(monkeypatch):
    for var, _ in rc.ENV_VARS_DB:
        monkeypatch.delenv(var, raising=False)
    assert rc.fetch_env_vars() == {"database": {}}
    monkeypatch.setenv("MOPT_DB_NAME", "n1")
    monkeypatch.setenv("ORION_DB_NAME", "n2")          # the first listed variable wins
    monkeypatch.setenv("ORION_DB_TYPE", "pickleddb")
    monkeypatch.setenv("MOPT_DB_ADDRESS", "/tmp/db.pkl")
    monkeypatch.setenv("MOPT_DB_PORT", "27017")
    assert rc.fetch_env_vars() == {"database": {"name": "n1", "type": "pickleddb",
                                                "host": "/tmp/db.pkl", "port": "27017"}}


@pytest.fixture
def script(tmp_path):
    p = tmp_path / "train.py"
    p.write_text("print(1)\n")
    return p


def test_metadata_version_and_user():
    md = rc.fetch_metadata({})
    assert md["orion_version"] and md["user"] and "user_script" not in md


def test_metadata_executable_script_is_absolute(script, monkeypatch):
    script.chmod(script.stat().st_mode | stat.S_IXUSR)
    monkeypatch.chdir(script.parent)
    md = rc.fetch_metadata({"user_args": ["train.py", "--lr~uniform(0,1)"]})
    assert md["user_script"] == str(script)
    assert md["user_args"] == ["--lr~uniform(0,1)"]


def test_metadata_non_executable_script_stays_relative(script, monkeypatch):
    monkeypatch.chdir(script.parent)
    md = rc.fetch_metadata({"user_args": ["train.py"]})
    assert md["user_script"] == "train.py" and md["user_args"] == []


def test_metadata_missing_script():
    with pytest.raises(OSError, match="does not exist"):
        rc.fetch_metadata({"user_args": ["/nonexistent/dir/train.py"]})


def test_metadata_empty_user_args():
    md = rc.fetch_metadata({"user_args": [""]})
    assert "user_script" not in md and "user_args" not in md


# ------------------------------------------------------------------ git metadata
def _git(cwd, *args):
    subprocess.run(["git", "-C", str(cwd), *args], check=True, capture_output=True,
                   env=dict(os.environ, GIT_AUTHOR_NAME="t", GIT_AUTHOR_EMAIL="t@t",
                            GIT_COMMITTER_NAME="t", GIT_COMMITTER_EMAIL="t@t"))


@pytest.fixture
def repo(tmp_path):
    _git(tmp_path, "init", "-q", "-b", "main")
    (tmp_path / "train.py").write_text("print(1)\n")
    _git(tmp_path, "add", "train.py")
    _git(tmp_path, "commit", "-q", "-m", "init")
    return tmp_path


def test_vcs_clean_repo(repo):
    vcs = rc.infer_versioning_metadata(str(repo / "train.py"))
    assert vcs["type"] == "git" and vcs["is_dirty"] is False
    assert len(vcs["HEAD_sha"]) == 40 and vcs["active_branch"] == "main"
    assert len(vcs["diff_sha"]) == 64


def test_vcs_dirty_repo_changes_the_diff_hash(repo):
    clean = rc.infer_versioning_metadata(str(repo / "train.py"))
    (repo / "train.py").write_text("print(2)\n")
    dirty = rc.infer_versioning_metadata(str(repo / "train.py"))
    assert dirty["is_dirty"] is True and dirty["diff_sha"] != clean["diff_sha"]
    assert dirty["HEAD_sha"] == clean["HEAD_sha"]


def test_vcs_detached_head(repo):
    sha = rc.infer_versioning_metadata(str(repo / "train.py"))["HEAD_sha"]
    _git(repo, "checkout", "-q", sha)
    vcs = rc.infer_versioning_metadata(str(repo / "train.py"))
    assert vcs["active_branch"] is None and vcs["HEAD_sha"] == sha


def test_vcs_outside_a_repo(tmp_path, caplog):
    p = tmp_path / "loose.py"
    p.write_text("")
    assert rc.infer_versioning_metadata(str(p)) == {}
    assert "not in a git repository" in caplog.text


def test_metadata_records_vcs(repo):
    md = rc.fetch_metadata({"user_args": [str(repo / "train.py")]})
    assert md["VCS"]["type"] == "git"


# ------------------------------------------------------------------ merge_configs
@pytest.mark.parametrize("configs,want", [
    (({"a": 1}, {"a": 2}), {"a": 2}),
    (({"a": 1}, {"a": 2}, {"a": 3}), {"a": 3}),
    (({"a": 1}, {"a": 2}, {"a": 3}, {"a": 4}), {"a": 4}),
    (({"a": 1}, {"b": 2}), {"a": 1, "b": 2}),
    (({"a": 1}, {"b": 2}, {"c": 3}), {"a": 1, "b": 2, "c": 3}),
    (({"a": 1}, {"b": 2}, {"c": 3}, {"d": 4}), {"a": 1, "b": 2, "c": 3, "d": 4}),
    (({"a": 1}, {"a": 2, "b": 2}), {"a": 2, "b": 2}),
    (({"a": 1}, {"a": 2, "b": 2}, {"b": 3, "c": 3}), {"a": 2, "b": 3, "c": 3}),
    (({"a": 1}, {"a": 2, "b": 2}, {"b": 3, "c": 3}, {"c": 4, "d": 4}),
     {"a": 2, "b": 3, "c": 4, "d": 4}),
])
def test_merge_flat(configs, want):
    assert rc.merge_configs(*[dict(c) for c in configs]) == want


def test_merge_nested_update():
    got = rc.merge_configs({"db": {"type": "ephemeral", "host": "h"}}, {"db": {"type": "mongo"}})
    assert got == {"db": {"type": "mongo", "host": "h"}}


def test_merge_nested_extend():
    got = rc.merge_configs({"db": {"type": "a"}}, {"db": {"port": 1}}, {"x": {"y": 2}})
    assert got == {"db": {"type": "a", "port": 1}, "x": {"y": 2}}


def test_merge_dict_replaces_scalar_and_scalar_replaces_dict():
    assert rc.merge_configs({"a": 1}, {"a": {"b": 2}}) == {"a": {"b": 2}}
    assert rc.merge_configs({"a": {"b": 2}}, {"a": 3}) == {"a": 3}


def test_merge_none_never_overwrites():
    assert rc.merge_configs({"a": 1, "b": {"c": 2}}, {"a": None, "b": {"c": None}}) == \
        {"a": 1, "b": {"c": 2}}


def test_merge_four_levels_of_precedence():
    default, env, file, cmd = ({"max_trials": 1, "db": {"type": "e"}}, {"db": {"type": "p"}},
                               {"max_trials": 5}, {"max_trials": 9, "name": "n"})
    assert rc.merge_configs(default, env, file, cmd) == {"max_trials": 9, "db": {"type": "p"},
                                                        "name": "n"}


# ------------------------------------------------------------------ Configuration
@pytest.fixture
def conf():
    c = Configuration()
    c.add_option("num", int, default=3, env_var="MOPT_TEST_NUM")
    c.add_option("ratio", float, default=0.5)
    c.add_option("name", str)
    c.add_option("flag", bool, default=False)
    sub = Configuration()
    sub.add_option("host", str, default="localhost")
    c.sub = sub
    return c


class TestConfiguration:
    def test_defaults(self, conf):
        assert conf.num == 3 and conf.ratio == 0.5 and conf.sub.host == "localhost"
        assert conf["sub.host"] == "localhost"

    def test_unset_without_default(self, conf):
        with pytest.raises(ConfigurationError, match="no default"):
            conf.name

    def test_unknown_option(self, conf):
        with pytest.raises(ConfigurationError, match="does not have"):
            conf.nope

    def test_set_typed_values(self, conf):
        conf.num = 7
        conf.ratio = 2
        conf.name = "x"
        assert (conf.num, conf.ratio, conf.name) == (7, 2.0, "x")

    def test_set_wrong_type(self, conf):
        with pytest.raises(TypeError):
            conf.num = "seven"

    def test_set_non_existing_option(self, conf):
        with pytest.raises(TypeError, match="add_option"):
            conf.other = 3

    def test_cannot_overwrite_option_with_subconfig(self, conf):
        with pytest.raises(TypeError):
            conf["num"] = Configuration()

    def test_dict_like_set(self, conf):
        conf["num"] = 11
        conf["sub.host"] = "h2"
        assert conf.num == 11 and conf.sub.host == "h2"

    def test_contains(self, conf):
        assert "num" in conf and "sub.host" in conf and "sub.port" not in conf
        assert "missing" not in conf

    def test_duplicate_option(self, conf):
        with pytest.raises(ValueError, match="already has"):
            conf.add_option("num", int)

    def test_bool_parsing(self, conf):
        conf.flag = "true"
        assert conf.flag is True

    def test_precedence_value_env_yaml_default(self, conf, tmp_path, monkeypatch):
        monkeypatch.delenv("MOPT_TEST_NUM", raising=False)
        y = tmp_path / "c.yaml"
        y.write_text("num: 4\nsub:\n  host: yh\n")
        conf.load_yaml(str(y))
        assert conf.num == 4 and conf.sub.host == "yh"          # yaml > default
        monkeypatch.setenv("MOPT_TEST_NUM", "5")
        assert conf.num == 5                                     # env > yaml
        conf.num = 6
        assert conf.num == 6                                     # value > env
        conf.unset("num")
        assert conf.num == 5

    def test_empty_yaml(self, conf, tmp_path):
        y = tmp_path / "e.yaml"
        y.write_text("")
        conf.load_yaml(str(y))
        assert conf.num == 3

    def test_yaml_unknown_key(self, conf, tmp_path):
        y = tmp_path / "u.yaml"
        y.write_text("bogus: 1\n")
        with pytest.raises(ConfigurationError):
            conf.load_yaml(str(y))

    def test_to_dict_and_defaults(self, conf, monkeypatch):
        monkeypatch.delenv("MOPT_TEST_NUM", raising=False)
        assert conf.to_dict() == {"num": 3, "ratio": 0.5, "flag": False,
                                  "sub": {"host": "localhost"}}
        assert conf.defaults()["sub"] == {"host": "localhost"}

    def test_env_vars_view(self, conf, monkeypatch):
        monkeypatch.setenv("MOPT_TEST_NUM", "8")
        assert conf.env_vars() == {"num": 8}
