"""Trial <-> point conversions (reference: ``src/orion/core/utils/format_trials.py:16-77``)."""
from __future__ import annotations

from ..core.trial import Trial


def trial_to_tuple(trial: Trial, space) -> tuple:
    params = {p.name: p.value for p in trial.params}
    if set(params) != set(space.keys()):
        raise ValueError(f"The trial {trial.id} has wrong params:\nTrial params: "
                         f"{sorted(params)}\nSpace dims: {sorted(space.keys())}")
    return tuple(params[name] for name in space.keys())


def tuple_to_trial(data, space) -> Trial:
    if len(data) != len(space):
        raise ValueError(f"point of length {len(data)} for a space of {len(space)} dimensions")
    params = [dict(name=dim.name, type=dim.type, value=data[i])
              for i, dim in enumerate(space.values())]
    return Trial(params=params)


def dict_to_trial(params: dict, space) -> Trial:
    return tuple_to_trial(tuple(params[k] for k in space.keys()), space)


def get_trial_results(trial: Trial) -> dict:
    """{'objective': lie or objective or None, 'constraint': [...], 'gradient': tuple|None}."""
    lie, objective = trial.lie, trial.objective
    out = {"objective": lie.value if lie else (objective.value if objective else None),
           "constraint": [r.value for r in trial.results if r.type == "constraint"]}
    grad = trial.gradient
    out["gradient"] = tuple(grad.value) if grad else None
    return out


def standard_param_name(name: str) -> str:
    return name.lstrip("/").lstrip("-").replace("-", "_")
