"""PathAnalyser: paths -> one instruction string (reference: PathAnalyser.py).

Host-side decision layer.  Restated step for step from
PathAnalyser.py:15-390, with one addition: the wall clock is injectable
(``clock``, default ``time.time``), because the reference's answer depends on
``time.time()`` (:335) and a 5 s instruction history (:375-382) -- a frozen
clock makes it reproducible (tests/test_surface.py checks the answers of 372
reference frames run with the same frozen clock).
"""
from __future__ import annotations

import time
from types import SimpleNamespace
from typing import Callable, ClassVar, Optional

import numpy as np

from .models import FinalAnswer, Instruction, Path

_TYPE_RANK = {"turn": 0, "curve": 0, "bearing": 1}
_DANGER_RANK = {"immediate": 0, "high": 1, "medium": 2, "low": 3}
# danger upgrades when a paired previous instruction turned by more than the threshold (:240-273)
_BEARING_UPGRADE = {"high": (12.5, "immediate"), "medium": (7.5, "high"), "low": (3.75, "medium")}
_TURN_UPGRADE = {"high": (15, "immediate"), "medium": (10, "high"), "low": (7.5, "medium")}
_PAIR_WINDOW_MS = 1500
_HISTORY_MS = 5000


class _HistRows:
    """One row per instruction of PathAnalyser.previous_instructions, in insertion order (keys non-decreasing):
    ts, bearing, distance, direction code, start x / y, danger rank, angle_change -- what _pairs tests and the
    upgrade reads.  History entries are not changed once stored (a call upgrades only its own instructions, before
    they are stored), so their rows stay exact.  Rows [n0, n) of growable arrays; front rows dropped by n0."""

    _F = (("ts", np.int64), ("bearing", np.bool_), ("dist", np.float64), ("dir", np.int64), ("sx", np.float64),
          ("sy", np.float64), ("rank", np.int64), ("angle", np.float64))

    def __init__(self, cap: int = 1024):
        self.a = {k: np.empty(cap, t) for k, t in self._F}
        self.n0 = self.n = 0
        self.codes: dict = {}
        self.last = None
        self._dict = None
        self._len = -1

    def code(self, direction) -> int:
        return self.codes.get(direction, -1)

    def matches(self, prev) -> bool:
        return self._dict is prev and self._len == len(prev)

    def sync(self, prev) -> None:
        self._dict, self._len = prev, len(prev)

    def append(self, ts: int, instructions) -> None:
        m = len(instructions)
        self.last = ts
        if m == 0:
            return
        cap = self.a["ts"].size
        if self.n + m > cap:
            live = self.n - self.n0
            ncap = max(cap, 2 * (live + m))
            for k, t in self._F:
                b = np.empty(ncap, t)
                b[:live] = self.a[k][self.n0:self.n]
                self.a[k] = b
            self.n0, self.n = 0, live
        i = self.n
        for j, ins in enumerate(instructions):
            r = i + j
            self.a["ts"][r] = ts
            self.a["bearing"][r] = ins.instruction_type == "bearing"
            self.a["dist"][r] = ins.distance
            self.a["dir"][r] = self.codes.setdefault(ins.direction, len(self.codes))
            self.a["sx"][r] = ins.start.x
            self.a["sy"][r] = ins.start.y
            self.a["rank"][r] = _DANGER_RANK[ins.danger]
            self.a["angle"][r] = ins.angle_change
        self.n += m

    def drop_ts(self, ts: int) -> None:
        """Drop the trailing rows of key ts (the newest entry, replaced)."""
        self.n = self.n0 + int(np.searchsorted(self.a["ts"][self.n0:self.n], ts, side="left"))

    def prune(self, oldest_kept_above: int) -> None:
        """Drop the rows with ts < oldest_kept_above (now - ts > the history span)."""
        self.n0 += int(np.searchsorted(self.a["ts"][self.n0:self.n], oldest_kept_above, side="left"))

    def window(self, above: int):
        """Views of the rows with ts > above (now - ts < the pair window)."""
        j = self.n0 + int(np.searchsorted(self.a["ts"][self.n0:self.n], above, side="right"))
        return SimpleNamespace(**{k: self.a[k][j:self.n] for k, _ in self._F})


class PathAnalyser:
    _instance: ClassVar[Optional["PathAnalyser"]] = None
    _initialized: bool = False

    def __new__(cls, *args, **kwargs):
        if cls._instance is None:
            cls._instance = super().__new__(cls)
        return cls._instance

    def __init__(self, clock: Callable[[], float] | None = None):
        if not self._initialized:
            self._initialized = True
            self.paths: list[Path] = []
            self.previous_instructions: dict[int, list[Instruction]] = {}
            self.instructions: list[Instruction] = []
            self.clock = clock or time.time
            self._rows = None  # _HistRows of previous_instructions (see _hist_rows)
        elif clock is not None:
            self.clock = clock

    # :35-77
    def _analyse_path(self, path: Path) -> Instruction | None:
        angle, length = path.angle, path.length
        if length < self.frame_height * 0.3:
            return None
        a = abs(angle)
        danger = "high" if a > 45 else "medium" if a > 25 else "low"
        kind = "bearing" if angle < 20 else "curve" if angle < 35 else "turn"
        if path.start.x == path.end.x:
            direction = "straight"
        else:
            direction = "left" if path.start.x > path.end.x else "right"
        return Instruction(direction=direction, danger=danger, distance=length, start=path.start, end=path.end,
                           angle_change=angle, length=length, instruction_type=kind)

    # :79-143
    def _analyse_corners(self, path: Path) -> list[Instruction]:
        out = []
        for corner in path.corners:
            dist = corner.start.y  # larger y = closer to the user
            if dist < self.frame_height * 0.5:
                continue
            h_mul = np.exp((np.log(2) / self.frame_height) * dist) - 1
            a_mul = np.exp((np.log(2) / 90) * abs(corner.angle_change)) - 1
            score = (h_mul * 0.7) + (a_mul * 0.3)
            if score > 0.75:
                danger = "immediate"
            elif score > 0.65:
                danger = "high"
            elif score > 0.45:
                danger = "medium"
            else:
                danger = "low"
            out.append(Instruction(direction=corner.direction, danger=danger, distance=dist, start=corner.start,
                                   end=corner.end, angle_change=corner.angle_change, length=corner.length,
                                   instruction_type="turn" if corner.sharpness == "sharp" else "curve"))
        return out

    def _analyse_instructions(self, instructions: list[Instruction]) -> list[Instruction]:  # :145-156 (identity)
        return instructions

    def _recent(self, previous, now):
        """The history entries a pair can come from (dt = now - ts < the pair window: both of the pair tests
        require it), in insertion order."""
        return [(ts, v) for ts, v in previous.items() if now - ts < _PAIR_WINDOW_MS]

    def _remember(self, now, instructions):
        """previous_instructions[now] = instructions, then the entries older than the 5 s history dropped
        (:375-382).  The reference rebuilds the dict per call; while the keys arrive in non-decreasing order the
        expired entries are a prefix, deleted from the front (same entries kept, same order), and the feature rows
        of _HistRows follow the dict."""
        hist = self._hist_rows()
        prev = self.previous_instructions
        if hist is not None and (not prev or now >= hist.last):
            if now in prev:  # the newest key again: its entry is replaced in place
                hist.drop_ts(now)
            prev[now] = instructions
            hist.append(now, instructions)
            while True:
                ts = next(iter(prev))
                if now - ts <= _HISTORY_MS:
                    break
                del prev[ts]
            hist.prune(now - _HISTORY_MS)
            hist.sync(prev)
            return
        prev[now] = instructions
        self.previous_instructions = {ts: v for ts, v in prev.items() if now - ts <= _HISTORY_MS}
        self._rows = None

    def _hist_rows(self):
        """The feature rows of previous_instructions, or None when its keys are not in non-decreasing insertion
        order (the literal scan then).  Rebuilt whenever the dict is not the one _remember last left (replaced or
        resized from outside, e.g. a test's reset)."""
        prev = self.previous_instructions
        h = self._rows
        if h is None or not h.matches(prev):
            keys = list(prev)
            if any(a > b for a, b in zip(keys, keys[1:])):
                self._rows = None
                return None
            h = self._rows = _HistRows()
            for ts, v in prev.items():
                h.append(ts, v)
            h.sync(prev)
        return h

    def _upgrade_fast(self, previous, current, now) -> bool:
        """_analyse_previous_instructions' danger upgrades (:185-273) from the feature rows: per current
        instruction the pairable rows of the pair window as one vectorised test (the five tests of _pairs, same
        float64 operations), then the upgrades folded over its pairs in history order -- the literal loop's
        result, since a pair changes only its own current instruction and the pair set is fixed before any upgrade.
        False (nothing done) when the rows do not apply: the literal loop runs instead."""
        if previous is not self.previous_instructions:
            return False
        hist = self._hist_rows()
        if hist is None or now < hist.last:
            return False
        w = hist.window(now - _PAIR_WINDOW_MS)
        if w.ts.size == 0:
            return True
        H, W = self.frame_height, self.frame_width
        weight = w.sy / H
        for c in current:
            # ~(p.distance > c.distance), not p.distance <= c.distance: the literal test's result for NaN too
            keep = ~(w.dist > c.distance) & (w.dir == hist.code(c.direction)) & (w.rank <= _DANGER_RANK[c.danger])
            if c.instruction_type != "bearing":
                keep &= ~w.bearing
            keep &= (np.abs(w.sy - c.start.y) * weight) < H * 0.2
            keep &= (np.abs(w.sx - c.start.x) * weight) < W * 0.2
            idx = np.flatnonzero(keep)
            if idx.size == 0:
                continue
            turned = np.abs(w.angle[idx] - c.angle_change)
            table = _BEARING_UPGRADE if c.instruction_type == "bearing" else _TURN_UPGRADE
            pos = 0
            while True:
                rule = table.get(c.danger)
                if rule is None:
                    break
                hit = np.flatnonzero(turned[pos:] > rule[0])
                if hit.size == 0:
                    break
                c.danger = rule[1]
                pos += int(hit[0]) + 1
        return True

    def _pairs(self, previous, current, now):
        """Previous/current instruction pairs that describe the same feature (:185-230)."""
        pairs = []
        for ts, prev_list in self._recent(previous, now):
            for p in prev_list:
                for c in current:
                    if p.instruction_type == "bearing" and c.instruction_type != "bearing":
                        continue
                    if p.distance > c.distance or p.direction != c.direction:
                        continue
                    dt = now - ts
                    dy = abs(p.start.y - c.start.y)
                    weight = p.start.y / self.frame_height
                    if not (dt < _PAIR_WINDOW_MS and (dy * weight) < self.frame_height * 0.2):
                        continue
                    dx = abs(p.start.x - c.start.x)
                    if not (dt < _PAIR_WINDOW_MS and (dx * weight) < self.frame_width * 0.2):
                        continue
                    if _DANGER_RANK[p.danger] - _DANGER_RANK[c.danger] > 0:
                        continue
                    pairs.append((p, c))
        return pairs

    # :158-284
    def _analyse_previous_instructions(self, previous_instructions, current_instructions, current_timestamp):
        if not previous_instructions:
            return current_instructions
        if not self._upgrade_fast(previous_instructions, current_instructions, current_timestamp):
            for p, c in self._pairs(previous_instructions, current_instructions, current_timestamp):
                turned = abs(p.angle_change - c.angle_change)
                table = _BEARING_UPGRADE if c.instruction_type == "bearing" else _TURN_UPGRADE
                rule = table.get(c.danger)
                if rule is not None and turned > rule[0]:
                    c.danger = rule[1]
        # drop low-danger / far non-bearings -- with the reference's remove-while-iterating (:276-282)
        for ins in current_instructions:
            if ins.instruction_type != "bearing":
                if ins.danger == "low":
                    current_instructions.remove(ins)
                elif ins.distance < self.frame_height * 0.33:
                    current_instructions.remove(ins)
        return current_instructions

    # :286-313
    def determine_final_instruction(self, instructions: list[Instruction]) -> FinalAnswer:
        if not instructions:
            return FinalAnswer.CONTINUE_FORWARD
        urgent = [i for i in instructions if i.danger == "immediate"]
        if urgent:
            return FinalAnswer.MOVE_LEFT if urgent[0].direction == "left" else FinalAnswer.MOVE_RIGHT
        if len(instructions) == 1 and instructions[0].instruction_type == "bearing":
            return FinalAnswer.CONTINUE_FORWARD
        first = instructions[0].direction
        if first == "left":
            return FinalAnswer.MOVE_LEFT
        if first == "right":
            return FinalAnswer.MOVE_RIGHT
        return FinalAnswer.CONTINUE_FORWARD

    # :316-386
    def __call__(self, frame_height: int, frame_width: int, paths: list[Path]) -> str:
        self.paths = paths
        self.frame_height = frame_height
        self.frame_width = frame_width
        self.instructions = []
        now = int(self.clock() * 1000)
        for path in self.paths:
            ins = self._analyse_path(path)
            if ins:
                self.instructions.append(ins)
            if path.corners:
                self.instructions.extend(self._analyse_corners(path))
        self.instructions = self._analyse_instructions(self.instructions)
        self.unfiltered_instructions = sorted(
            self.instructions, key=lambda i: (_TYPE_RANK[i.instruction_type], _DANGER_RANK[i.danger]))
        self.filtered_instructions = self._analyse_previous_instructions(self.previous_instructions,
                                                                          self.instructions, now)
        self._remember(now, self.unfiltered_instructions)
        return self.determine_final_instruction(self.filtered_instructions).value


path_analyser = PathAnalyser()
