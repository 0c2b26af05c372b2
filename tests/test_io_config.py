"""Configuration precedence, command-line parsing/templating, prior extraction from the command
line and from YAML / JSON / generic text config files, and per-trial rendering (reference:
tests/unittests/core/io/test_config.py, test_cmdline_parser.py, test_orion_cmdline_parser.py,
test_converters.py -- behaviour re-specified, not copied)."""
import json
import os

import pytest
import yaml

from metaopt_amd.core.config import Configuration, ConfigurationError, define_config
from metaopt_amd.core.trial import Trial
from metaopt_amd.io.cmdline_parser import CmdlineParser
from metaopt_amd.io.convert import (GenericConverter, JSONConverter, YAMLConverter,
                                    infer_converter_from_file_type)
from metaopt_amd.io.space_parser import SpaceCmdlineParser


# ------------------------------------------------------------------ Configuration
class TestConfiguration:
    def _cfg(self):
        c = Configuration()
        c.add_option("port", int, 27017, env_var="MOPT_TEST_PORT")
        c.add_option("name", str)
        sub = Configuration()
        sub.add_option("heartbeat", int, 120)
        c.worker = sub
        return c

    def test_default_env_yaml_value_precedence(self, tmp_path, monkeypatch):
        c = self._cfg()
        assert c.port == 27017
        p = tmp_path / "c.yaml"
        p.write_text(yaml.safe_dump({"port": 1000, "worker": {"heartbeat": 5}}))
        c.load_yaml(str(p))
        assert c.port == 1000 and c.worker.heartbeat == 5
        monkeypatch.setenv("MOPT_TEST_PORT", "2000")
        assert c.port == 2000                     # env > yaml
        c.port = 3000
        assert c.port == 3000                     # value > env
        c.unset("port")
        assert c.port == 2000

    def test_types_are_enforced(self):
        c = self._cfg()
        with pytest.raises(TypeError):
            c.port = "not-an-int"
        c.port = "42"
        assert c.port == 42

    def test_missing_and_unknown(self):
        c = self._cfg()
        with pytest.raises(ConfigurationError):
            c.name
        with pytest.raises(ConfigurationError):
            c.nope
        with pytest.raises(ValueError):
            c.add_option("port", int)
        with pytest.raises(TypeError):
            c.newkey = 3

    def test_dotted_access_and_contains(self):
        c = self._cfg()
        c["worker.heartbeat"] = 7
        assert c["worker.heartbeat"] == 7 and "worker.heartbeat" in c and "worker.x" not in c
        assert c.to_dict()["worker"] == {"heartbeat": 7}

    def test_unknown_yaml_key_raises(self, tmp_path):
        c = self._cfg()
        p = tmp_path / "bad.yaml"
        p.write_text("bogus: 1\n")
        with pytest.raises(ConfigurationError):
            c.load_yaml(str(p))

    def test_global_schema(self, monkeypatch):
        cfg = define_config()
        assert cfg.worker.heartbeat == 120 and cfg.worker.max_broken == 3
        assert cfg.worker.max_idle_time == 60 and cfg.database.port == 27017
        monkeypatch.setenv("ORION_DB_TYPE", "mongodb")   # reference env var names work too
        assert cfg.database.type == "mongodb"
        assert cfg.env_vars()["database"] == {"type": "mongodb"}


# ------------------------------------------------------------------ CmdlineParser
class TestCmdlineParser:
    def test_parse_kinds(self, tmp_path):
        f = tmp_path / "data.txt"
        f.write_text("x")
        p = CmdlineParser()
        args = p.parse(["train.py", "--lr=0.1", "--flag", "-v", "3", "--multi", "a", "b",
                        "--path", str(f)])
        assert args["_pos_0"] == "train.py" and args["lr"] == "0.1"
        assert args["flag"] is True and args["v"] == "3" and args["multi"] == ["a", "b"]
        assert args["path"] == os.path.abspath(str(f))

    def test_template_roundtrip(self):
        p = CmdlineParser()
        p.parse(["script", "--aa", "1", "--bb", "x", "y", "--cc", "-d", "2"])
        out = p.format({"_pos_0": "script", "aa": 5, "bb": ["p", "q"], "cc": True, "d": 3})
        assert out == ["script", "--aa", "5", "--bb", "p", "q", "--cc", "-d", "3"]
        q = CmdlineParser()
        q.set_state_dict(p.get_state_dict())
        assert q.format({"_pos_0": "s", "aa": 1, "bb": ["u", "v"], "d": 0}) == \
            ["s", "--aa", "1", "--bb", "u", "v", "--cc", "-d", "0"]

    def test_duplicate_and_reparse(self):
        with pytest.raises(ValueError):
            CmdlineParser().parse(["--a", "1", "--a", "2"])
        p = CmdlineParser()
        p.parse(["--a", "1"])
        with pytest.raises(RuntimeError):
            p.parse(["--a", "1"])


# ------------------------------------------------------------------ converters
class TestConverters:
    def test_infer(self, tmp_path):
        assert isinstance(infer_converter_from_file_type("a.yaml"), YAMLConverter)
        assert isinstance(infer_converter_from_file_type("a.yml"), YAMLConverter)
        assert isinstance(infer_converter_from_file_type("a.json"), JSONConverter)
        assert isinstance(infer_converter_from_file_type("a.cfg"), GenericConverter)

    def test_yaml_json_roundtrip(self, tmp_path):
        data = {"a": {"b": 1, "c": [1, 2]}, "d": "x"}
        for conv, name in ((YAMLConverter(), "f.yaml"), (JSONConverter(), "f.json")):
            path = str(tmp_path / name)
            conv.generate(path, data)
            assert conv.parse(path) == data

    def test_generic_parse_and_generate(self, tmp_path):
        src = tmp_path / "model.cfg"
        src.write_text("lr = lr~loguniform(1e-5, 1.0)\nlayers {n: /arch/n~randint(1, 4)}\n"
                       "keep = 3\n")
        conv = GenericConverter()
        parsed = conv.parse(str(src))
        assert parsed == {"lr": "loguniform(1e-5, 1.0)", "arch": {"n": "randint(1, 4)"}}
        out = tmp_path / "inst.cfg"
        conv.generate(str(out), {"lr": 0.01, "arch": {"n": 3}})
        assert out.read_text() == "lr = 0.01\nlayers {n: 3}\nkeep = 3\n"
        clone = GenericConverter()
        clone.set_state_dict(json.loads(json.dumps(conv.get_state_dict())))
        clone.generate(str(out), {"lr": 0.5, "arch": {"n": 1}})
        assert out.read_text().startswith("lr = 0.5\n")

    def test_generic_namespace_conflict(self, tmp_path):
        src = tmp_path / "bad.cfg"
        src.write_text("a~uniform(0, 1)\na~uniform(0, 2)\n")
        with pytest.raises(ValueError):
            GenericConverter().parse(str(src))


# ------------------------------------------------------------------ prior extraction
def _trial(**params):
    return Trial(params=[{"name": k, "type": "real", "value": v} for k, v in params.items()])


class TestSpaceCmdlineParser:
    def test_command_line_priors(self):
        p = SpaceCmdlineParser()
        p.parse(["train.py", "--lr~loguniform(1e-5, 1.0)", "-x~uniform(-1, 1)", "--epochs", "3",
                 "--out~/abs/path"])
        assert p.priors == {"/lr": "loguniform(1e-5, 1.0)", "/x": "uniform(-1, 1)"}
        out = p.format(trial=_trial(**{"/lr": 0.01, "/x": 0.5}))
        assert out[:3] == ["train.py", "--lr", "0.01"] and "-x" in out and "0.5" in out
        assert "--out~/abs/path" in out           # a path after '~' is not a prior

    def test_branching_markers_are_priors(self):
        p = SpaceCmdlineParser()
        p.parse(["s.py", "--new~+uniform(0, 1)", "--old~-", "--a~>b"])
        assert p.priors == {"/new": "+uniform(0, 1)", "/old": "-", "/a": ">b"}

    @pytest.mark.parametrize("ext", ["yaml", "json"])
    def test_config_file_priors_and_instantiation(self, tmp_path, ext):
        data = {"optim": {"lr": "orion~loguniform(1e-4, 1)", "name": "sgd"},
                "layers": ["orion~choices([1, 2])", 7]}
        path = tmp_path / f"conf.{ext}"
        (YAMLConverter() if ext == "yaml" else JSONConverter()).generate(str(path), data)
        p = SpaceCmdlineParser()
        p.parse(["train.py", "--config", str(path), "--seed~randint(0, 9)"])
        assert p.priors == {"/optim/lr": "loguniform(1e-4, 1)", "/layers/0": "choices([1, 2])",
                            "/seed": "randint(0, 9)"}
        with pytest.raises(ValueError):
            p.format(trial=_trial(**{"/optim/lr": 0.1}))     # needs a config path
        inst = tmp_path / f"trial.{ext}"
        out = p.format(str(inst), _trial(**{"/optim/lr": 0.1, "/layers/0": 2, "/seed": 4}))
        assert out == ["train.py", "--config", str(inst), "--seed", "4"]
        got = (YAMLConverter() if ext == "yaml" else JSONConverter()).parse(str(inst))
        assert got == {"optim": {"lr": 0.1, "name": "sgd"}, "layers": [2, 7]}

    def test_duplicate_between_file_and_cmdline(self, tmp_path):
        path = tmp_path / "c.yaml"
        YAMLConverter().generate(str(path), {"lr": "orion~uniform(0, 1)"})
        with pytest.raises(ValueError):
            SpaceCmdlineParser().parse(["s", "--config", str(path), "--lr~uniform(0, 1)"])

    def test_trial_and_experiment_templates(self):
        p = SpaceCmdlineParser()
        p.parse(["s.py", "--xx~uniform(0, 1)", "--ckpt", "{trial.working_dir}/m.pt",
                 "--name", "{exp.name}"])
        t = _trial(**{"/xx": 0.25})
        t.working_dir = "/tmp/wd"

        class Exp:
            name = "exp-a"
        out = p.format(trial=t, experiment=Exp())
        assert out == ["s.py", "--xx", "0.25", "--ckpt", "/tmp/wd/m.pt", "--name", "exp-a"]

    def test_state_dict_roundtrip(self, tmp_path):
        path = tmp_path / "c.yaml"
        YAMLConverter().generate(str(path), {"a": "orion~uniform(0, 1)"})
        p = SpaceCmdlineParser()
        p.parse(["s", "--config", str(path), "--b~uniform(0, 2)"])
        q = SpaceCmdlineParser()
        q.set_state_dict(json.loads(json.dumps(p.get_state_dict())))
        assert q.priors == p.priors
        inst = tmp_path / "i.yaml"
        assert q.format(str(inst), _trial(**{"/a": 0.5, "/b": 1.5})) == \
            p.format(str(inst), _trial(**{"/a": 0.5, "/b": 1.5}))
