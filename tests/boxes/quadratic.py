#!/usr/bin/env python3
"""Black box of the functional tests: f(x) = 4 (x - 34.56789)^2 + 23.4 with gradient, scaled by
noise that vanishes at full fidelity (the reference's demo/algos black boxes' objective)."""
import argparse
import random

from metaopt_amd.client import report_results


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-x", type=float, required=True)
    ap.add_argument("-y", type=float, default=None)
    ap.add_argument("-z", type=float, default=None)
    ap.add_argument("--fidelity", type=int, default=10)
    ap.add_argument("--noise", action="store_true", help="noisy below full fidelity")
    args = ap.parse_args()
    d = args.x - 34.56789
    if args.noise:
        d *= random.gauss(0, (1 - args.fidelity / 10) + 0.0001)
    report_results([{"name": "example_objective", "type": "objective", "value": 4 * d * d + 23.4},
                    {"name": "example_gradient", "type": "gradient", "value": [8 * d]}])


if __name__ == "__main__":
    main()
