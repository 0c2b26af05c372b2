"""``mopt db test`` stages (the behaviour the reference pins in
tests/unittests/core/cli/test_checks.py): presence of the default / environment / file
configuration, creation of the backend, and the write / read / count / remove round trip, each
passing, skipping or failing as documented.  Written against this package's API."""
import pytest

from metaopt_amd.cli.db import test as checks
from metaopt_amd.storage.database import PickledDB
from metaopt_amd.utils.exceptions import CheckError


@pytest.fixture
def presence():
    return checks.PresenceStage({})


def _cfg(tmp_path, text):
    p = tmp_path / "c.yaml"
    p.write_text(text)
    return str(p)


def test_default_config_pass(presence):
    assert presence.check_default_config() == ("Success", "")
    assert set(presence.db_config) == {"type", "name", "host", "port"}


def test_env_vars_pass(presence, monkeypatch):
    monkeypatch.setenv("MOPT_DB_TYPE", "ephemeraldb")
    presence.check_default_config()
    assert presence.check_environment_vars() == ("Success", "")
    assert presence.db_config["type"] == "ephemeraldb"


def test_env_vars_skip(presence, monkeypatch):
    for var in ("MOPT_DB_TYPE", "MOPT_DB_NAME", "MOPT_DB_ADDRESS", "MOPT_DB_PORT",
                "ORION_DB_TYPE", "ORION_DB_NAME", "ORION_DB_ADDRESS", "ORION_DB_PORT"):
        monkeypatch.delenv(var, raising=False)
    assert presence.check_environment_vars() == ("Skipping", "No environment variables found.")


def test_config_file_pass(tmp_path):
    stage = checks.PresenceStage({"config": _cfg(tmp_path, "database:\n  type: ephemeraldb\n")})
    stage.check_default_config()
    assert stage.check_configuration_file() == ("Success", "")
    assert stage.db_config["type"] == "ephemeraldb"


def test_config_file_missing(presence):
    assert presence.check_configuration_file() == ("Skipping", "No configuration file found.")


def test_config_file_without_database(tmp_path):
    stage = checks.PresenceStage({"config": _cfg(tmp_path, "name: x\n")})
    assert stage.check_configuration_file() == ("Skipping",
                                                 "No database found in configuration file.")


def test_config_file_database_without_values(tmp_path):
    stage = checks.PresenceStage({"config": _cfg(tmp_path, "database:\n  other: 1\n")})
    assert stage.check_configuration_file() == (
        "Skipping", "No configuration value found inside `database`.")


def test_post_stage_prints_the_configuration(presence, capsys):
    presence.check_default_config()
    presence.post_stage()
    assert "Using configuration:" in capsys.readouterr().out


def test_creation_pass(tmp_path):
    presence = checks.PresenceStage({})
    presence.db_config = {"type": "pickleddb", "host": str(tmp_path / "db.pkl")}
    creation = checks.CreationStage(presence)
    assert creation.check_database_creation() == ("Success", "")
    assert isinstance(creation.instance, PickledDB)


def test_creation_fails_for_unknown_backend():
    presence = checks.PresenceStage({})
    presence.db_config = {"type": "nosuchdb"}
    with pytest.raises(CheckError, match="nosuchdb"):
        checks.CreationStage(presence).check_database_creation()


@pytest.fixture
def operations(tmp_path):
    presence = checks.PresenceStage({})
    presence.db_config = {"type": "pickleddb", "host": str(tmp_path / "db.pkl")}
    creation = checks.CreationStage(presence)
    creation.check_database_creation()
    return checks.OperationsStage(creation)


def test_operations_round_trip(operations):
    for check in operations.checks():
        assert check() == ("Success", "")
    assert operations.db.count("test") == 0


def test_read_fails_without_document(operations):
    with pytest.raises(CheckError, match="Expected to read"):
        operations.check_read()


def test_count_fails_on_unexpected_count(operations):
    operations.check_write()
    operations.check_write()
    with pytest.raises(CheckError, match="Expected 1 document, found 2"):
        operations.check_count()


def test_remove_fails_when_documents_stay(operations, monkeypatch):
    operations.check_write()
    monkeypatch.setattr(operations.db, "remove", lambda *a, **k: 0)
    with pytest.raises(CheckError, match="Expected 0 document"):
        operations.check_remove()


def test_main_reports_every_check(tmp_path, capsys, monkeypatch):
    monkeypatch.setenv("MOPT_DB_TYPE", "pickleddb")
    monkeypatch.setenv("MOPT_DB_ADDRESS", str(tmp_path / "m.pkl"))
    assert checks.main({}) == 0
    out = capsys.readouterr().out
    for name in ("default config", "environment vars", "configuration file",
                 "database creation", "write", "read", "count", "remove"):
        assert f"{name}..." in out


def test_main_stops_at_the_first_failure(capsys, monkeypatch):
    monkeypatch.setenv("MOPT_DB_TYPE", "nosuchdb")
    assert checks.main({}) == 1
    out = capsys.readouterr().out
    assert "database creation... Failure" in out and "write..." not in out
