"""Fault injection for recovery tests ("a fault-injection flag ... for
contract tests", "RCCL communicator re-init on rank failure").

``NGA_FAULT`` holds comma-separated rules ``<action>@<where>`` where ``where`` is a
colon-joined filter of ``rank<N>``, ``step<N>`` (engine step / follower step counter) and
``site<name>`` (``driver``, ``follower``). Actions:

* ``crash`` — ``os._exit(71)`` (a dead rank: RCCL peers block, torchrun's elastic agent tears
  the group down and restarts it with fresh communicators);
* ``hang``  — sleep forever (a wedged rank: the driver's fail-fast watchdog turns it into a
  crash after ``watchdog_s``);
* ``raise`` — ``RuntimeError`` (an in-process step failure: streams get an error frame, the
  server keeps serving).

Rules fire only in the first incarnation of an elastic job (``TORCHELASTIC_RESTART_COUNT``
is 0 or unset) unless ``NGA_FAULT_ALWAYS=1``, so a restarted group comes back healthy.
Example: ``NGA_FAULT=crash@rank1:step5`` kills TP rank 1 at its fifth step.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import List, Optional


@dataclass
class Rule:
    action: str
    rank: Optional[int] = None
    step: Optional[int] = None
    site: Optional[str] = None

    def matches(self, rank: int, step: int, site: str) -> bool:
        return ((self.rank is None or self.rank == rank) and (self.step is None or self.step == step)
                and (self.site is None or self.site == site))


def parse(spec: str) -> List[Rule]:
    rules = []
    for part in filter(None, (p.strip() for p in spec.split(","))):
        action, _, where = part.partition("@")
        if action not in ("crash", "hang", "raise"):
            raise ValueError(f"unknown fault action {action!r} in NGA_FAULT")
        r = Rule(action)
        for f in filter(None, where.split(":")):
            if f.startswith("rank"):
                r.rank = int(f[4:])
            elif f.startswith("step"):
                r.step = int(f[4:])
            elif f.startswith("site"):
                r.site = f[4:]
            else:
                raise ValueError(f"unknown fault filter {f!r} in NGA_FAULT")
        rules.append(r)
    return rules


class FaultInjector:
    def __init__(self, spec: Optional[str] = None, rank: Optional[int] = None):
        spec = os.environ.get("NGA_FAULT", "") if spec is None else spec
        first = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") in ("", "0")
        active = first or os.environ.get("NGA_FAULT_ALWAYS") == "1"
        self.rules = parse(spec) if (spec and active) else []
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else rank

    def __bool__(self) -> bool:
        return bool(self.rules)

    def check(self, step: int, site: str) -> None:
        for r in self.rules:
            if r.matches(self.rank, step, site):
                if r.action == "crash":
                    os._exit(71)
                if r.action == "hang":
                    while True:
                        time.sleep(3600)
                raise RuntimeError(f"injected fault at step {step} ({site}, rank {self.rank})")
