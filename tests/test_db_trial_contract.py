"""Document-database and Trial contracts (the behaviour the reference pins in
tests/unittests/core/test_ephemeraldb.py, test_pickleddb.py and test_trial.py): queries with
operators and dotted keys, projections, upserts and atomic read-and-write, unique and compound
indexes, removal, the same semantics through the file-backed PickledDB; trial ids, statuses,
typed results and the document round trip.  Written against this package's API."""
import pytest

from metaopt_amd.core.trial import Trial
from metaopt_amd.storage.database import DuplicateKeyError, EphemeralDB, PickledDB

DOCS = [{"_id": 1, "a": 1, "b": {"x": 2}}, {"_id": 2, "a": 2, "b": {"x": 3}}, {"_id": 3, "a": 3}]


@pytest.fixture(params=["ephemeral", "pickled"])
def db(request, tmp_path):
    d = EphemeralDB() if request.param == "ephemeral" else PickledDB(host=str(tmp_path / "x.pkl"))
    d.write("c", [dict(x) for x in DOCS])
    return d


def _ids(docs):
    return sorted(d["_id"] for d in docs)


class TestQueries:
    def test_insert_count(self, db):
        assert db.count("c") == 3 and db.count("c", {"a": 2}) == 1

    def test_equality_and_dotted_keys(self, db):
        assert _ids(db.read("c", {"a": 1})) == [1]
        assert _ids(db.read("c", {"b.x": 3})) == [2]
        assert db.read("c", {"b.x": 99}) == []

    def test_subdocument_equality(self, db):
        assert _ids(db.read("c", {"b": {"x": 2}})) == [1]

    @pytest.mark.parametrize("query,ids", [
        ({"a": {"$gte": 2}}, [2, 3]), ({"a": {"$gt": 2}}, [3]), ({"a": {"$lt": 2}}, [1]),
        ({"a": {"$lte": 2}}, [1, 2]), ({"a": {"$ne": 2}}, [1, 3]), ({"a": {"$in": [1, 3]}}, [1, 3]),
        ({"a": {"$nin": [1]}}, [2, 3]), ({"a": {"$gt": 1, "$lte": 3}}, [2, 3]),
    ])
    def test_operators(self, db, query, ids):
        assert _ids(db.read("c", query)) == ids

    def test_unsupported_operator(self, db):
        with pytest.raises(ValueError, match="not supported"):
            db.read("c", {"a": {"$regex": "x"}})

    def test_projection_keeps_id_unless_excluded(self, db):
        got = db.read("c", {"a": {"$gte": 2}}, selection={"a": 1})
        assert sorted(got, key=lambda d: d["_id"]) == [{"a": 2, "_id": 2}, {"a": 3, "_id": 3}]
        assert sorted(d["a"] for d in db.read("c", {}, selection={"_id": 0, "a": 1})) == [1, 2, 3]
        assert all(set(d) == {"a"} for d in db.read("c", {}, selection={"_id": 0, "a": 1}))

    def test_results_are_copies(self, db):
        doc = db.read("c", {"a": 1})[0]
        doc["a"] = 100
        assert db.count("c", {"a": 100}) == 0

    def test_unknown_collection_is_empty(self, db):
        assert db.read("nothing", {}) == [] and db.count("nothing") == 0


class TestWrites:
    def test_update_by_query(self, db):
        assert db.write("c", {"z": 9}, query={"a": 1}) == 1
        assert db.read("c", {"a": 1})[0]["z"] == 9 and db.count("c") == 3

    def test_update_many(self, db):
        assert db.write("c", {"flag": True}, query={"a": {"$gte": 2}}) == 2
        assert db.count("c", {"flag": True}) == 2

    def test_update_nothing(self, db):
        assert db.write("c", {"z": 1}, query={"a": 42}) == 0

    def test_read_and_write_returns_the_new_document(self, db):
        got = db.read_and_write("c", {"a": 2}, {"a": 20})
        assert got["_id"] == 2 and got["a"] == 20
        assert db.count("c", {"a": 20}) == 1

    def test_read_and_write_no_match(self, db):
        assert db.read_and_write("c", {"a": 99}, {"a": 20}) is None

    def test_remove(self, db):
        assert db.remove("c", {"a": {"$gte": 2}}) == 2 and db.count("c") == 1

    def test_remove_nothing(self, db):
        assert db.remove("c", {"a": 77}) == 0 and db.count("c") == 3

    def test_insert_duplicate_id(self, db):
        with pytest.raises(DuplicateKeyError):
            db.write("c", {"_id": 1, "a": 5})


class TestIndexes:
    def test_unique_index(self, db):
        db.ensure_index("c", "a", unique=True)
        assert "a_1" in db.index_information("c")
        with pytest.raises(DuplicateKeyError):
            db.write("c", {"_id": 4, "a": 3})

    def test_unique_index_on_update(self, db):
        db.ensure_index("c", "a", unique=True)
        with pytest.raises(DuplicateKeyError):
            db.write("c", {"a": 1}, query={"_id": 2})

    def test_compound_index(self, db):
        db.ensure_index("c", [("a", 1), ("z", 1)], unique=True)
        assert "a_1_z_1" in db.index_information("c")
        db.write("c", {"_id": 5, "a": 1, "z": 2})          # (1, 2) differs from (1, None)

    def test_drop_index(self, db):
        db.ensure_index("c", "a", unique=True)
        db.drop_index("c", "a_1")
        assert "a_1" not in db.index_information("c")
        db.write("c", {"_id": 4, "a": 3})                  # no longer unique

    def test_id_index_always_present(self, db):
        assert "_id_" in db.index_information("c")

    def test_index_on_nonunique_data_refused(self, db):
        db.write("c", {"_id": 9, "a": 1})
        with pytest.raises(DuplicateKeyError):
            db.ensure_index("c", "a", unique=True)


class TestPickledPersistence:
    def test_survives_reopen(self, tmp_path):
        path = str(tmp_path / "p.pkl")
        PickledDB(host=path).write("c", {"_id": 1, "v": 3})
        assert PickledDB(host=path).read("c", {"_id": 1})[0]["v"] == 3

    def test_indexes_survive_reopen(self, tmp_path):
        path = str(tmp_path / "p.pkl")
        a = PickledDB(host=path)
        a.write("c", {"_id": 1, "v": 3})
        a.ensure_index("c", "v", unique=True)
        with pytest.raises(DuplicateKeyError):
            PickledDB(host=path).write("c", {"_id": 2, "v": 3})


# ------------------------------------------------------------------ Trial
def _trial(**kw):
    params = [dict(name="/x", type="real", value=0.5), dict(name="/c", type="categorical",
                                                           value="a")]
    return Trial(experiment=kw.pop("experiment", "e1"), params=params, **kw)


class TestTrial:
    def test_defaults(self):
        t = _trial()
        assert t.status == "new" and t.results == [] and t.objective is None
        assert t.params_dict == {"/x": 0.5, "/c": "a"}

    def test_id_is_md5_of_params_and_experiment(self):
        t = _trial()
        assert len(t.id) == 32 and t.id == _trial().id
        assert t.id != _trial(experiment="e2").id
        assert t.hash_name == t.id

    def test_params_order_is_part_of_the_identity(self):
        a = _trial()
        b = Trial(experiment="e1", params=list(reversed(a.to_dict()["params"])))
        assert a.id != b.id

    def test_params_repr_and_names(self):
        t = _trial()
        assert t.params_repr() == "/x:0.5,/c:a"
        assert t.full_name == ".x:0.5-.c:a"
        assert t.arguments == {"x": 0.5, "c": "a"}

    def test_typed_results(self):
        t = _trial()
        t.results = [dict(name="o", type="objective", value=1.0),
                     dict(name="g", type="gradient", value=[1, 2]),
                     dict(name="s", type="statistic", value=3),
                     dict(name="c", type="constraint", value=0.1)]
        assert t.objective.value == 1.0 and t.gradient.value == [1, 2]
        assert [r.name for r in t.statistics] == ["s"]
        assert [r.name for r in t.constraints] == ["c"] and t.lie is None

    def test_bad_status(self):
        with pytest.raises(ValueError, match="not one of"):
            _trial().status = "bogus"

    @pytest.mark.parametrize("status", Trial.allowed_stati)
    def test_every_allowed_status(self, status):
        t = _trial()
        t.status = status
        assert t.status == status

    def test_bad_result_type(self):
        with pytest.raises(ValueError, match="not one of"):
            _trial().results = [dict(name="o", type="weird", value=1.0)]

    def test_unknown_attribute(self):
        with pytest.raises(AttributeError):
            Trial(bogus=1)

    def test_document_roundtrip(self):
        t = _trial()
        t.results = [dict(name="o", type="objective", value=2.0)]
        d = t.to_dict()
        assert {"_id", "experiment", "params", "results", "status", "parents"} <= set(d)
        back = Trial(**d)
        assert back.id == t.id and back.objective.value == 2.0

    def test_build_from_documents(self):
        d = _trial().to_dict()
        built = Trial.build([d, d])
        assert len(built) == 2 and all(b.id == d["_id"] for b in built)

    def test_str(self):
        assert str(_trial()) == "Trial(experiment='e1', status='new', params=/x:0.5,/c:a)"

    def test_working_dir(self):
        t = _trial()
        t.working_dir = "/tmp/w"
        assert t.working_dir == "/tmp/w"
