"""``orion.client``: the user-script API, re-exported from :mod:`metaopt_amd.client`."""
from metaopt_amd.client import (IS_ORION_ON, RESULTS_FILENAME, Study,  # noqa: F401
                                insert_trials, register, report_results)
