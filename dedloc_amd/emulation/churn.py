"""Churn schedule: scripted drop-out / drop-in of a peer (spot preemption, volunteers leaving).

Grammar (``--churn_schedule``): comma-separated events ``[MODE@]AT[s]:DURATION``

* ``AT``       global collaborative step at which the event fires; with an ``s`` suffix, seconds since
               the peer started training.
* ``DURATION`` seconds the peer stays away.
* ``MODE``     ``leave`` (default): the peer stops training and reporting (its progress record expires
               after ``metadata_expiration``, so the others re-plan without it), then rejoins and
               re-synchronises through ``load_state_from_peers``.
               ``restart``: like a preempted spot instance that is respawned — the peer also DROPS
               its parameters, optimizer state and step counter and must download them on return.

Example: ``leave@5:20,restart@120s:30``.  These are IN-PROCESS events.  Real process-level churn
— a SIGKILLed trainer (spot preemption, no clean-up) replaced by a brand-new process with a new
peer id, the reference's respawn loop (``AWS_runner.ipynb:342-370``) — is the launcher's
``--kill_schedule`` / ``--respawn`` (``cli/launch_collaboration.py``; tested in
``tests/test_launcher_churn.py``).  Both work because no peer belongs to a launch-time world: every
averaging group builds its communicators through the DHT (``parallel/comm.py``).
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from typing import List, Optional

_EVENT_RE = re.compile(r"^\s*(?:(leave|restart)@)?(\d+(?:\.\d+)?)(s?)\s*:\s*(\d+(?:\.\d+)?)\s*$")


@dataclass
class ChurnEvent:
    at: float
    duration: float
    mode: str = "leave"
    in_seconds: bool = False
    fired: bool = False


def parse_churn_schedule(spec: Optional[str]) -> List[ChurnEvent]:
    if not spec:
        return []
    events = []
    for item in spec.split(","):
        if not item.strip():
            continue
        m = _EVENT_RE.match(item)
        if m is None:
            raise ValueError(f"bad churn event {item!r}; expected [leave|restart@]AT[s]:DURATION")
        mode, at, sec, dur = m.groups()
        events.append(ChurnEvent(at=float(at), duration=float(dur), mode=mode or "leave", in_seconds=sec == "s"))
    return events


class ChurnController:
    def __init__(self, events: List[ChurnEvent], start_time: float):
        self.events = events
        self.start_time = start_time

    def due(self, global_step: int, now: float) -> Optional[ChurnEvent]:
        """The first not-yet-fired event whose trigger has passed (each event fires once)."""
        for ev in self.events:
            if ev.fired:
                continue
            hit = (now - self.start_time >= ev.at) if ev.in_seconds else (global_step >= ev.at)
            if hit:
                ev.fired = True
                return ev
        return None
