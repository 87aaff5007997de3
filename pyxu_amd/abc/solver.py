"""
Iterative-solver engine (mirrors reference ``pyxu.abc.solver``, src/pyxu/abc/solver.py:26-718).

Same execution modes (BLOCK / ASYNC / MANUAL), stop/log/writeback rates, history records, worker
thread, exception capture and ``data.npz`` checkpoint format.  The math state lives on the MI355X;
device -> host copies happen only at stop-criterion evaluations and at writeback.
"""
import datetime as dt
import enum
import logging
import operator
import os
import pathlib as plib
import shutil
import sys
import tempfile
import threading

import numpy as np

import pyxu_amd.runtime as pxrt
from pyxu_amd.util import to_NUMPY

__all__ = ["Mode", "Solver", "StoppingCriterion"]


def _on_device(v):
    return getattr(getattr(v, "device", None), "type", "cpu") != "cpu"


_SAVE_LOCK = threading.Lock()


def _atomic_savez(path, arrays):
    """np.savez into a temporary file of its own in the same folder, then rename over `path`.  Writers
    (the caller's writeback() and the asynchronous checkpoint thread) are serialised, and each writes
    its own temporary file, so a rename never moves a half-written file over `path`."""
    path = plib.Path(path)
    with _SAVE_LOCK:
        fd, tmp = tempfile.mkstemp(dir=path.parent, prefix=path.name + ".", suffix=".tmp")
        try:
            with os.fdopen(fd, "wb") as f:
                np.savez(f, **arrays)
            os.replace(tmp, path)
        except BaseException:
            try:
                os.unlink(tmp)
            except OSError:
                pass
            raise


@enum.unique
class Mode(enum.Enum):
    BLOCK = enum.auto()
    MANUAL = enum.auto()
    ASYNC = enum.auto()


class StoppingCriterion:
    """State machine deciding when to stop (solver.py:37-94); compose with ``&`` / ``|``."""

    def stop(self, state) -> bool:
        raise NotImplementedError

    def stop_async(self, state):
        """Two-phase stop(): enqueue the device work of the decision now, return a callable that
        completes it (same decision, same info()).  Default: decide now."""
        r = self.stop(state)
        return lambda: r

    def info(self) -> dict:
        raise NotImplementedError

    def clear(self):
        pass

    def __or__(self, other):
        return _StoppingCriteriaComposition(lhs=self, rhs=other, op=operator.or_)

    def __and__(self, other):
        return _StoppingCriteriaComposition(lhs=self, rhs=other, op=operator.and_)


class _StoppingCriteriaComposition(StoppingCriterion):
    def __init__(self, lhs, rhs, op):
        self._lhs, self._rhs, self._op = lhs, rhs, op

    def stop(self, state) -> bool:
        return self._op(self._lhs.stop(state), self._rhs.stop(state))

    def stop_async(self, state):
        lhs, rhs = self._lhs.stop_async(state), self._rhs.stop_async(state)
        return lambda: self._op(lhs(), rhs())

    def info(self):
        return {**self._lhs.info(), **self._rhs.info()}

    def clear(self):
        self._lhs.clear()
        self._rhs.clear()


_NULL_LOGGER = logging.getLogger("pyxu_amd.internal_solver")
_NULL_LOGGER.addHandler(logging.NullHandler())
_NULL_LOGGER.propagate = False


class Solver:
    """Base class of iterative solvers (solver.py:97-718)."""

    def __init__(self, *, folder=None, exist_ok=False, stop_rate=1, writeback_rate=None, verbosity=None,
                 show_progress=True, log_var=frozenset(), _internal=False):
        self._mstate = dict()
        self._astate = dict(history=None, idx=0, log_rate=None, log_var=None, logger=None, stdout=None, stop_crit=None,
                            stop_rate=None, track_objective=None, wb_rate=None, workdir=None, mode=None, active=None,
                            worker=None, internal=bool(_internal), lock=threading.RLock())
        try:
            if _internal:  # sub-solver of an operator method (QuadraticFunc.prox): no workdir / log / checkpoint
                pass
            elif folder is None:
                folder = plib.Path(tempfile.mkdtemp(prefix="pyxu_amd_"))
            elif (folder := plib.Path(folder).expanduser().resolve()).exists() and (not exist_ok):
                raise FileExistsError(f"{folder} already exists.")
            else:
                shutil.rmtree(folder, ignore_errors=True)
                folder.mkdir(parents=True)
            self._astate["workdir"] = folder
        except FileExistsError:
            raise
        except Exception:
            raise Exception(f"folder: expected path-like, got {type(folder)}.")
        try:
            assert stop_rate >= 1
            self._astate["stop_rate"] = int(stop_rate)
        except Exception:
            raise ValueError(f"stop_rate must be positive, got {stop_rate}.")
        try:
            self._astate["wb_rate"] = writeback_rate
            if writeback_rate is not None:
                assert writeback_rate % self._astate["stop_rate"] == 0
                self._astate["wb_rate"] = int(writeback_rate)
        except Exception:
            raise ValueError(f"writeback_rate must be a multiple of stop_rate({stop_rate}), got {writeback_rate}.")
        try:
            if verbosity is None:
                verbosity = self._astate["stop_rate"]
            assert verbosity % self._astate["stop_rate"] == 0
            self._astate["log_rate"] = int(verbosity)
            self._astate["stdout"] = bool(show_progress)
        except Exception:
            raise ValueError(f"verbosity must be a multiple of stop_rate({stop_rate}), got {verbosity}.")
        if isinstance(log_var, str):
            log_var = (log_var,)
        self._astate["log_var"] = frozenset(log_var)

    # ------------------------------------------------------------------ public API
    def fit(self, **kwargs):
        from pyxu_amd import profile

        profile.instrument(self)  # PXA_PROFILE roctx ranges / PXA_DEBUG_SYNC checks around m_step
        prof = profile.enabled()
        if prof:
            profile.range_push(f"{type(self).__name__}.fit")
        try:
            self._fit_init(
                mode=kwargs.pop("mode", Mode.BLOCK),
                stop_crit=kwargs.pop("stop_crit", None),
                track_objective=kwargs.pop("track_objective", False),
            )
            self.m_init(**kwargs)
            self._fit_run()
        finally:
            if prof:
                profile.range_pop()

    def m_init(self, **kwargs):
        raise NotImplementedError

    def m_step(self):
        raise NotImplementedError

    def steps(self, n=None):
        self._check_mode(Mode.MANUAL)
        i = 0
        plan = self._lag_plan()
        if plan is not None:  # lagged stop checks: the same items, _LAG checks behind the device
            gen = self._lag_loop(plan)
            ended = False
            try:
                while (n is None) or (i < n):
                    try:
                        item = next(gen)
                    except StopIteration:
                        ended = True
                        break
                    yield item
                    i += 1
            finally:
                if not ended:
                    gen.close()
                    self._lag_settle()
            if ended:
                self._astate["mode"] = None
                self._wb_drain()
                self._cleanup_logger()
            return
        while (n is None) or (i < n):
            if self._step():
                # == stats()[0]; the history concatenation of stats() is O(#records) per step and its
                # result is discarded here (reference solver.py:378 computes and drops it)
                yield {k: self._mstate.get(k) for k in self._astate["log_var"]}
                i += 1
            else:
                self._astate["mode"] = None
                self._wb_drain()  # checkpoints of this run are on disk when steps() returns
                self._cleanup_logger()
                return

    def stats(self):
        # ASYNC: the worker thread appends and flushes records concurrently; the records lock keeps
        # pending -> history moves atomic, so no record is dropped, duplicated or reordered
        with self._astate["lock"]:
            self._flush_records()
            history = self._astate["history"]
            if history is not None:
                history = np.concatenate(history, dtype=history[0].dtype, axis=0) if len(history) > 0 else None
        logical = self._astate.get("lag_logical")
        if logical is not None:  # MANUAL mode under the lagged engine: the state of the last item steps() yielded
            return dict(logical), history
        data = {k: self._mstate.get(k) for k in self._astate["log_var"]}
        return data, history

    @property
    def workdir(self):
        return self._astate["workdir"]

    @property
    def logfile(self):
        return self.workdir / "solver.log"

    @property
    def datafile(self):
        return self.workdir / "data.npz"

    def busy(self) -> bool:
        self._check_mode(Mode.ASYNC, Mode.BLOCK)
        return self._astate["active"].is_set()

    def solution(self):
        raise NotImplementedError

    def stop(self):
        self._check_mode(Mode.ASYNC, Mode.BLOCK)
        self._astate["active"].clear()
        self._astate["worker"].join()
        self._astate.update(mode=None, active=None, worker=None)
        self._wb_drain()
        self._cleanup_logger()

    def writeback(self):
        """Checkpoint ``log_var`` + history to ``workdir/data.npz`` (solver.py:562-570).  Synchronous:
        earlier asynchronous checkpoints are drained first, so the file holds this state on return."""
        if self._astate.get("internal"):
            return
        self._wb_drain()
        data, history = self.stats()
        kwargs = {k: to_NUMPY(v) for (k, v) in dict(history=history, **data).items() if (v is not None)}
        _atomic_savez(self.datafile, kwargs)

    def _writeback_async(self):
        """Mid-run checkpoint (``writeback_rate``) without stalling the device queue: the ``log_var``
        arrays are snapshotted on the device (pxa_copy2d into fresh buffers, ordered on the solver's
        stream before the next m_step) and a writer thread waits for that snapshot's event, copies it
        to the host and writes ``data.npz`` (checkpoints land in iteration order; the file is replaced
        atomically, so a reader never sees a partial checkpoint)."""
        if self._astate.get("internal"):
            return
        from pyxu_amd import _dev

        data, history = self.stats()
        snap, ev = {}, None
        for k, v in data.items():
            if v is None:
                continue
            if _on_device(v):
                c = _dev.empty_like(v)
                n = v.numel()
                if n:
                    _dev.copy2d(v.contiguous(), c, 1, n, n, n)
                snap[k] = c
            else:
                snap[k] = np.array(v, copy=True)
        if any(_on_device(v) for v in snap.values()):
            import torch

            ev = torch.cuda.Event()
            _dev.record_event(ev)
        prev = self._astate.get("wb_thread")
        ast = self._astate

        def job():
            if prev is not None:
                prev.join()
            try:
                if ev is not None:
                    ev.synchronize()
                kwargs = {k: to_NUMPY(v) for (k, v) in dict(history=history, **snap).items() if (v is not None)}
                _atomic_savez(self.datafile, kwargs)
            except Exception as e:  # surfaced by the next synchronous writeback
                ast["wb_error"] = e

        t = threading.Thread(target=job, name="pyxu_amd-writeback", daemon=True)
        t.start()
        ast["wb_thread"] = t

    def _wb_drain(self):
        t = self._astate.pop("wb_thread", None)
        if t is not None:
            t.join()
        e = self._astate.pop("wb_error", None)
        if e is not None:
            raise e

    def default_stop_crit(self):
        raise NotImplementedError("No default stopping criterion defined.")

    def objective_func(self):
        raise NotImplementedError("No objective function defined.")

    def _solve_inline(self, stop_crit=None, **kwargs):
        """Run m_init and the stop/m_step loop on the calling thread (the iterates and stop decisions are
        those of ``fit()``).  Used for sub-solvers created inside operator methods (QuadraticFunc.prox -> CG,
        operator.py:1273-1291), where the reference's per-fit temporary folder, log file, worker thread, final
        checkpoint and iteration history are side effects nobody reads: they cost milliseconds per call
        against a sub-millisecond iteration on the device (the history flush alone ~40 us between ADMM's
        x-update and the rest of its step)."""
        from pyxu_amd import profile

        profile.instrument(self)
        self._mstate.clear()
        if stop_crit is None:
            stop_crit = self.default_stop_crit()
        stop_crit.clear()
        self._astate.update(history=[], pending=[], idx=0, logger=_NULL_LOGGER, stop_crit=stop_crit,
                            track_objective=False, mode=Mode.MANUAL, active=None, worker=None, exception=None)
        self.m_init(**kwargs)
        while self._step():
            pass
        self._astate["mode"] = None
        if self._astate.get("exception") is not None:
            raise self._astate["exception"]

    # ------------------------------------------------------------------ internals
    def _fit_init(self, mode, stop_crit, track_objective):
        def _init_logger():
            logger = logging.getLogger(str(self.workdir))
            logger.handlers.clear()
            logger.setLevel("DEBUG")
            fmt = logging.Formatter(fmt="{levelname} -- {message}", style="{")
            handlers = [logging.FileHandler(self.logfile, mode="w")]
            if (mode is Mode.BLOCK) and self._astate["stdout"]:
                handlers.append(logging.StreamHandler(sys.stdout))
            for h in handlers:
                h.setLevel("DEBUG")
                h.setFormatter(fmt)
                logger.addHandler(h)
            logger.propagate = False
            logger._pxa_direct = list(handlers)  # the record log lines may bypass LogRecord (_log_lines)
            return logger

        self._mstate.clear()
        if stop_crit is None:
            stop_crit = self.default_stop_crit()
        stop_crit.clear()
        if track_objective:
            from pyxu_amd.opt.stop import Memorize

            stop_crit |= Memorize(var="objective_func")
        self._astate.update(history=[], pending=[], idx=0, logger=_init_logger(), stop_crit=stop_crit,
                            track_objective=track_objective, mode=mode, active=None, worker=None)

    def _fit_run(self):
        mode = self._astate["mode"]
        if mode is Mode.MANUAL:
            return
        self._astate.update(active=threading.Event(), worker=Solver._Worker(self))
        self._astate["active"].set()
        self._astate["worker"].start()
        if mode is Mode.BLOCK:
            self._astate["worker"].join()
            self.stop()

    def _check_mode(self, *modes):
        m = self._astate["mode"]
        if m not in modes:
            if m is None:
                raise ValueError("Illegal method call: invoke Solver.fit() first.")
            raise ValueError("Illegal method call: can only be used if Solver.fit() invoked with mode=Any["
                             + ", ".join(_.name for _ in modes) + "]")

    # ---- speculative stop checks: the next m_step runs on the device while the host decides
    def _spec_supported(self) -> bool:
        """True when m_step can be undone (`_spec_begin` / `_spec_rollback`): solvers override."""
        return False

    def _spec_begin(self):
        raise NotImplementedError

    def _spec_rollback(self, token):
        raise NotImplementedError

    def _step_speculative(self, idx, _ml, log_on) -> bool:
        """A stop check whose decision does not stall the device queue: the criterion enqueues its
        statistics (stop_async), m_step is launched speculatively, then the decision is read.  If it
        says stop, m_step is undone (the state is the one the check saw) and the solver ends exactly as
        the synchronous path would: same iterates, same history records, same log lines."""
        ast = self._astate
        resolve = ast["stop_crit"].stop_async(self._mstate)
        token = self._spec_begin()
        err = None
        ast["idx"] += 1  # as on the synchronous path: m_step sees the index of the step after it
        try:
            self.m_step()
        except Exception as e:  # raised only if the check says continue (then the reference calls m_step)
            err = e
        # the host would now wait for the decision while the device runs the previous step: write deferred
        # history records / log lines meanwhile, _SPEC_BATCH at a time (one structured array and one write per
        # batch: at stop_rate 1 the host, not the device, bounds the step, and one record per check cost
        # ~5 us of it; r05d host profile)
        if len(ast["pending"]) >= self._SPEC_BATCH:
            with ast["lock"]:
                if len(ast["pending"]) >= self._SPEC_BATCH:
                    items = ast["pending"][: self._SPEC_BATCH]
                    del ast["pending"][: self._SPEC_BATCH]
                    # unflushed at most _RECORD_LAG lines: a reader of solver.log lags by at most one batch
                    n = ast.get("unflushed", 0) + len(items)
                    ast["unflushed"] = 0 if n >= self._RECORD_LAG else n
                    self._record_batch(items, flush=n >= self._RECORD_LAG)
        if resolve():
            ast["idx"] -= 1
            self._spec_rollback(token)
            with ast["lock"]:
                self._flush_records()
                self._record(idx, ast["stop_crit"].info(), dt.datetime.now(), pxrt.getPrecision().value, log_on)
            if log_on:
                ast["logger"].info(f"[{dt.datetime.now()}] Stopping Criterion satisfied -> END")
            self.writeback()
            return False
        if err is None and ast["mode"] is not Mode.ASYNC:
            # continue: the device has one step of work left, so the next launch is what matters now.  The
            # check's history record is captured after it (_take_capture: before anything that can change the
            # criterion's info(), i.e. the next check, and after the next launch otherwise).  ASYNC mode
            # captures now: stats() may run on another thread.
            ast["capture"] = (idx, _ml and log_on)
            return True
        rec = (idx, ast["stop_crit"].info(), dt.datetime.now(), pxrt.getPrecision().value, _ml and log_on)
        with ast["lock"]:
            ast["pending"].append(rec)
        if err is not None:
            raise err
        return True

    def _take_capture(self):
        """History record of a speculative check whose capture was deferred past the next launch."""
        ast = self._astate
        cap = ast.pop("capture", None)
        if cap is not None:
            rec = (cap[0], ast["stop_crit"].info(), dt.datetime.now(), pxrt.getPrecision().value, cap[1])
            with ast["lock"]:
                ast["pending"].append(rec)

    def _step(self) -> bool:
        ast = self._astate
        idx = ast["idx"]
        _ms = idx % ast["stop_rate"] == 0
        _ml = idx % ast["log_rate"] == 0
        _mw = (ast["wb_rate"] is not None) and (idx % ast["wb_rate"] == 0)

        log_on = not ast.get("internal")
        if "capture" in ast and (_ms or _mw):  # before this step's check can change the criterion's info()
            self._take_capture()
        if ast["pending"] and (_mw or idx - ast["pending"][0][0] >= self._RECORD_LAG):
            self._flush_records()

        try:
            if _ms and ast["track_objective"]:
                self._mstate["objective_func"] = self.objective_func().reshape(-1)
            if _ms and not _mw and self._spec_supported():
                return self._step_speculative(idx, _ml, log_on)
            if _ms and ast["stop_crit"].stop(self._mstate):
                if not ast.get("internal"):  # (an inline sub-solve keeps no history: nobody can read it)
                    with ast["lock"]:
                        self._flush_records()
                        self._record(idx, ast["stop_crit"].info(), dt.datetime.now(), pxrt.getPrecision().value,
                                     log_on)
                if log_on:
                    ast["logger"].info(f"[{dt.datetime.now()}] Stopping Criterion satisfied -> END")
                self.writeback()
                return False
            if _mw:  # the checkpoint saves the pre-step state: keep the reference order (solver.py:626-652)
                with ast["lock"]:
                    self._record(idx, ast["stop_crit"].info() if _ms else None, dt.datetime.now(),
                                 pxrt.getPrecision().value, _ml and log_on)
                self._writeback_async()
                ast["idx"] += 1
                self.m_step()
                return True
            # m_step is enqueued first, so the device starts on it right after the stop decision.  This
            # iteration's history record and log line (solver.py:604-624) are captured after the launch
            # (info() reads only the stop criterion, which m_step does not touch; the log time stamp is
            # taken here) and written a few steps later, when the device queue holds enough work to hide
            # them (_flush_records: before the next stop check / log / checkpoint and in stats()).  The
            # records are the reference's, also when m_step raises.
            ast["idx"] += 1
            try:
                self.m_step()
            finally:
                if "capture" in ast:
                    self._take_capture()
                if (_ms or (_ml and log_on)) and not ast.get("internal"):
                    rec = (idx, ast["stop_crit"].info() if _ms else None, dt.datetime.now(),
                           pxrt.getPrecision().value, _ml and log_on)
                    with ast["lock"]:
                        ast["pending"].append(rec)
            return True
        except Exception as e:
            self._on_exception(e)
            return False

    def _on_exception(self, e):
        """The reference's handling of an exception raised by a step (solver.py:626-652): records and log lines
        written, the message to stderr and the log, the exception kept for the caller."""
        ast = self._astate
        self._flush_records()
        self._flush_log()  # lines written unflushed by speculative checks reach the file first
        msg = f"[{dt.datetime.now()}] Something went wrong -> EXCEPTION RAISED"
        if ast.get("internal"):
            ast["exception"] = e
            return
        print("\n".join([msg, f"More information: {self.logfile}."]), file=sys.stderr)
        try:  # the "last valid checkpoint" below is on disk once the writer is drained
            self._wb_drain()
        except Exception:
            pass
        if ast["wb_rate"] is not None:
            _, r = divmod(ast["idx"], ast["wb_rate"])
            msg = "\n".join([msg, f"Last valid checkpoint done at iteration={ast['idx'] - r}."])
        ast["logger"].exception(msg, exc_info=e)
        ast["exception"] = e

    # ---- lagged stop checks: at stop_rate 1 the speculative check above still makes the host wait, every step, for
    # the statistics of the step before (~28 us of Python plus the flag round trip against ~30 us of device work per
    # step: the loop was host-bound, r05v).  The lagged engine keeps up to _LAG checks unresolved instead: each check
    # is enqueued (its statistics folded by the device into a ring of host flag buffers) and the next step launched
    # at once; checks are resolved in order as their statistics land.  The state at every unresolved check is held
    # (references: the solver never writes a tensor it still references), so when check j says stop, the steps
    # launched after it are dropped and the solver ends in the state of check j.  Decisions, iterates, history
    # records, log lines, MaxIter counts and steps() items are the synchronous path's (tests/test_gpu_solver_lag.py).
    # Applies to stop_rate 1 in BLOCK / MANUAL mode with an OR of MaxIter and one fused-path RelError, no
    # checkpoints, no objective tracking, and a solver that can restore a check's state (_lag_supported).
    _LAG = int(os.environ.get("PXA_STOP_LAG", "8"))
    # the fused RelError statistics folded by the step kernel's last workgroup (no fold launch) under the lagged
    # engine, where the host reads them several steps later anyway (PXA_LAG_INKERNEL=0: the fold launch)
    _LAG_INKERNEL = os.environ.get("PXA_LAG_INKERNEL", "0") == "1"
    # the statistics of check k computed by the launch of step k + 2 from the (x, x_prev) pair it reads anyway
    # (pxa_pgd_tv2d_plan_step_wfold) instead of by step k + 1's epilogue from an extra load of x: the same sums of the
    # same terms in another order, so the RelError values may differ from the synchronous path's in the last bits
    # (PXA_LAG_WINDOW=0: the epilogue statistics, bit-identical history)
    _LAG_WINDOW = os.environ.get("PXA_LAG_WINDOW", "1") == "1"
    _LAG_RECORDS = 4  # deferred history records written per batch by the lagged engine
    _LAG_MAX_BYTES = int(float(os.environ.get("PXA_LAG_MAX_BYTES", str(16 * 2**30))))  # iterates held in flight

    def _lag_supported(self) -> bool:
        return False

    def _lag_snapshot(self):
        """The state a check sees, restorable by _lag_restore (solvers override)."""
        raise NotImplementedError

    def _lag_restore(self, snap, undone):
        """Return to the state `snap` of a check; `undone` m_steps launched after it are dropped."""
        raise NotImplementedError

    def _lag_flush(self):
        """Make every enqueued check's statistics land without a further m_step (solvers whose steps publish the
        statistics of an earlier check override)."""

    def _lag_plan(self):
        """(RelError leaf, MaxIter leaves) when the lagged engine applies to this run, else None."""
        from pyxu_amd.opt import stop as pxst

        ast = self._astate
        if (self._LAG < 1 or ast.get("stop_rate") != 1 or ast.get("wb_rate") is not None or ast.get("track_objective")
                or ast.get("internal") or ast.get("mode") not in (Mode.BLOCK, Mode.MANUAL) or not self._lag_supported()):
            return None
        leaves = []

        def walk(c):
            if isinstance(c, _StoppingCriteriaComposition):
                return c._op is operator.or_ and walk(c._lhs) and walk(c._rhs)
            leaves.append(c)
            return True

        if not walk(ast["stop_crit"]):
            return None
        rels = [c for c in leaves if type(c) is pxst.RelError]
        maxs = [c for c in leaves if type(c) is pxst.MaxIter]
        if len(rels) != 1 or len(rels) + len(maxs) != len(leaves):
            return None
        r = rels[0]
        if r._var not in ast["log_var"] or r._norm != 2 or r._f is not pxst._identity or r._reduce is not None:
            return None
        # the held states of the checks in flight: at most ~(_LAG + 3) iterates of the size of `var` at once
        v = self._mstate.get(r._var)
        nbytes = int(v.numel()) * int(v.element_size()) if hasattr(v, "numel") else 0
        if nbytes * (self._LAG + 3) > self._LAG_MAX_BYTES:
            return None
        return r, maxs

    class _LagCheck:
        __slots__ = ("idx", "resolve", "pre", "snap", "stamp", "log", "ready", "counts", "rel_prev", "post", "info")

    def _lag_loop(self, plan):
        """Generator running the fit to its end: yields the synchronous path's steps() item once per check that did
        not stop (so BLOCK mode just drains it), up to _LAG checks behind the launches."""
        import collections

        rel, maxs = plan
        ast, mst = self._astate, self._mstate
        crit = ast["stop_crit"]
        depth = self._LAG
        rel._nbufs = depth + 3  # flag buffers: the checks in flight, the one being resolved, the next launch's
        rel._in_kernel_fold = self._LAG_INKERNEL
        log_on = not ast.get("internal")
        prec = pxrt.getPrecision().value
        pend = collections.deque()
        ast["lag"] = pend
        win = self._LAG_WINDOW
        try:
            while True:
                idx = ast["idx"]
                e = Solver._LagCheck()
                e.idx, e.snap, e.rel_prev = idx, self._lag_snapshot(), rel._x_prev
                # window statistics need a next launch: not for the check at which MaxIter ends the run
                last = False  # MaxIter ends the run at this check
                for m in maxs:
                    last = last or m._i + 1 > m._n
                rel._window_stats = win and not last
                e.resolve = crit.stop_async(mst)
                e.pre = crit.info()  # MaxIter counts of this check (the RelError value is filled in when resolved)
                e.counts = [m._i for m in maxs]
                kind, probe = getattr(rel, "_last_async", ("sync", None))
                e.ready = probe if kind == "fused" else (lambda: True)  # ("event": drained below)
                e.stamp, e.log = dt.datetime.now(), (idx % ast["log_rate"] == 0) and log_on
                e.post = e.info = None
                pend.append(e)
                if kind == "event" or last:  # (OR composite: MaxIter's stop() above returned True exactly when `last`)
                    self._lag_flush()
                    drain = len(pend)  # a one-buffer statistic, or the last check: resolve everything now
                else:
                    ast["idx"] += 1
                    self.m_step()
                    e.post = {k: mst.get(k) for k in ast["log_var"]}
                    drain = 0
                    # deferred records: written while the host would otherwise spin on the oldest check (the queue is
                    # full and its statistics have not landed), else a few per launch once a backlog builds up (one
                    # batch of _RECORD_LAG would stall a queue that a host synchronisation has just drained: ~0.1 ms of
                    # host work against one step of device work)
                    npr = len(ast["pending"])
                    if npr > 0:
                        if len(pend) > depth and pend[0].ready is not None and not pend[0].ready():
                            self._lag_records(min(npr, 2 * self._LAG_RECORDS))
                        elif npr >= 4 * self._LAG_RECORDS:
                            self._lag_records(self._LAG_RECORDS)
                free = 1  # at most one ready check per launch beyond the forced ones: the device queue stays fed (a run
                # of ready checks resolved back to back, e.g. after a host synchronisation, would leave it idle)
                while pend and (drain > 0 or len(pend) > depth or (free > 0 and pend[0].ready is not None and pend[0].ready())):
                    if drain <= 0 and len(pend) <= depth:
                        free -= 1
                    drain -= 1
                    c = pend.popleft()
                    stopped = c.resolve()
                    c.info = {**c.pre, **rel.info()}
                    if stopped:
                        self._lag_end(c, rel, maxs, pend, prec)
                        return
                    with ast["lock"]:
                        ast["pending"].append((c.idx, c.info, c.stamp, prec, c.log))
                    if c.post is None:  # (an "event" check resolved before its step: launch it now)
                        ast["idx"] += 1
                        self.m_step()
                        c.post = {k: mst.get(k) for k in ast["log_var"]}
                    ast["lag_logical"] = c.post if ast["mode"] is Mode.MANUAL else None
                    yield c.post
        except Exception as err:
            pend.clear()
            ast.pop("lag", None)
            ast.pop("lag_logical", None)
            self._on_exception(err)
        finally:
            rel._window_stats = False

    def _lag_records(self, k):
        """Write the oldest k deferred records (flushing the log every _RECORD_LAG records)."""
        ast = self._astate
        with ast["lock"]:
            items = ast["pending"][:k]
            del ast["pending"][:k]
            n = ast.get("unflushed", 0) + len(items)
            ast["unflushed"] = 0 if n >= self._RECORD_LAG else n
            self._record_batch(items, flush=n >= self._RECORD_LAG)

    def _lag_end(self, c, rel, maxs, pend, prec):
        """Check c said stop: drop the launches after it, restore its state, write its record, end the run."""
        ast = self._astate
        undone = ast["idx"] - c.idx
        pend.clear()
        ast.pop("lag", None)
        self._lag_restore(c.snap, undone)
        ast["idx"] = c.idx
        for m, n in zip(maxs, c.counts):
            m._i = n
        ast.pop("lag_logical", None)
        log_on = not ast.get("internal")
        with ast["lock"]:
            self._flush_records()
            self._record(c.idx, c.info, c.stamp, prec, c.log)
        if log_on:
            ast["logger"].info(f"[{dt.datetime.now()}] Stopping Criterion satisfied -> END")
        self.writeback()

    def _lag_settle(self):
        """steps() closed before the run ended: back to the state of its last item (the unresolved checks and
        the steps launched after it dropped; their MaxIter counts and RelError reference undone)."""
        ast = self._astate
        ast.pop("lag_logical", None)
        pend = ast.pop("lag", None)
        plan = self._lag_plan()
        if not pend or plan is None:
            return
        rel, maxs = plan
        k = pend[0]
        self._lag_restore(k.snap, ast["idx"] - k.idx)
        ast["idx"] = k.idx
        for m, n in zip(maxs, k.counts):
            m._i = n - 1
        rel._x_prev = k.rel_prev
        pend.clear()

    # steps between an iteration and the write of its deferred history record / log line: records and log
    # lines are written in batches (one structured array and one file write per batch), also at stop_rate 1
    _RECORD_LAG = 32
    _SPEC_BATCH = 16  # deferred records written per batch by the speculative stop checks

    def _record(self, it, data, stamp, ftype, log):
        """Append the history record of iteration `it` (stop-criterion info `data`, None = no record) and
        write its log line (solver.py:604-624)."""
        self._record_batch([(it, data, stamp, ftype, log)])

    def _record_batch(self, items, flush=True):
        """_record() for a run of deferred records, in order: consecutive records of one layout become one
        structured array (the history is a list of arrays that stats() concatenates), and their log lines
        are written with one call per handler (same text as one logger.info() per record)."""
        ast = self._astate
        cache = ast.setdefault("_hist_dtype", {})
        hist = ast["history"]
        msgs = []
        run, run_dtype = [], None
        run_logs = []  # (index in run of the record the line shows, iteration, stamp)

        def line(stamp, it, names, values):
            return "\n".join([f"[{stamp}] Iteration {it:>_d}"] + [f"\t{f}: {v}" for f, v in zip(names, values)])

        def close_run():
            # one structured array per run of same-layout records; the run's log lines are formatted from its
            # columns as Python scalars (f"{v}" of a NumPy scalar is f"{v.item()}": same text as record by record,
            # at a third of the cost -- at stop_rate 1 every step writes one)
            if run:
                names = run_dtype.names
                try:
                    arr = np.array(run, dtype=run_dtype)
                    cols = [arr[n].tolist() for n in names] if run_logs else None
                except (TypeError, ValueError):  # non-scalar info() values: field by field, as numpy assigns them
                    arr = np.zeros(len(run), dtype=run_dtype)
                    for i, r in enumerate(run):
                        for name, v in zip(names, r):
                            arr[i][name] = v
                    cols = None
                hist.append(arr)
                for k, it, stamp in run_logs:
                    msgs.append(line(stamp, it, names, [c[k] for c in cols] if cols is not None else arr[k]))
                run.clear()
                run_logs.clear()

        for it, data, stamp, ftype, log in items:
            if data is not None:
                key = (ftype, tuple(data))
                dtype = cache.get(key)
                if dtype is None:
                    dtype = cache[key] = np.dtype([("iteration", np.int64)] + [(k, ftype) for k in data])
                if dtype is not run_dtype:
                    close_run()
                    run_dtype = dtype
                run.append((it, *data.values()))
            if log:  # the line shows the newest history record
                if run:
                    run_logs.append((len(run) - 1, it, stamp))
                else:
                    h = hist[-1][-1]
                    msgs.append(line(stamp, it, h.dtype.names, h))
        close_run()
        if msgs:
            self._log_lines(msgs, flush)

    def _log_lines(self, msgs, flush=True):
        """logger.info(m) for each m: the solver's own handlers (``{levelname} -- {message}``, _init_logger) get
        the formatted text in one write per batch (flushed unless `flush` is False: the next batch, stats() or
        the end of the run flushes it); any other logger goes through logging."""
        logger = self._astate["logger"]
        handlers = getattr(logger, "_pxa_direct", None)
        if handlers is None or handlers != logger.handlers or not logger.isEnabledFor(logging.INFO):
            for m in msgs:
                logger.info(m)
            return
        text = "".join(f"INFO -- {m}\n" for m in msgs)
        for h in handlers:
            with h.lock:
                if h.stream is None and isinstance(h, logging.FileHandler):
                    h.stream = h._open()
                h.stream.write(text)
                if flush:
                    h.flush()
        if flush:
            self._astate["unflushed"] = 0

    def _flush_log(self):
        for h in getattr(self._astate.get("logger"), "_pxa_direct", None) or ():
            with h.lock:
                if h.stream is not None:
                    h.flush()
        self._astate["unflushed"] = 0

    def _flush_records(self):
        ast = self._astate
        if "capture" in ast:
            self._take_capture()
        if ast.get("pending"):
            with ast["lock"]:
                items, ast["pending"] = ast["pending"], []
                self._record_batch(items)

    def _cleanup_logger(self):
        logger = logging.getLogger(str(self.workdir))
        for handler in logger.handlers:
            handler.close()

    class _Worker(threading.Thread):
        def __init__(self, solver):
            super().__init__()
            self.slvr = solver
            # the worker must launch on the caller's device and stream (torch keeps both per thread)
            import torch

            self._dev = torch.cuda.current_device() if torch.cuda.is_available() else None
            self._stream = torch.cuda.current_stream() if torch.cuda.is_available() else None

        def run(self):
            import torch

            if self._dev is not None:
                torch.cuda.set_device(self._dev)
                with torch.cuda.stream(self._stream):
                    self._loop()
            else:
                self._loop()

        def _loop(self):
            plan = self.slvr._lag_plan()
            if plan is not None:
                for _ in self.slvr._lag_loop(plan):
                    if not self.slvr.busy():  # (not reached in BLOCK mode: the lagged engine runs to the end)
                        break
            else:
                while self.slvr.busy() and self.slvr._step():
                    pass
            self.slvr._astate["active"].clear()
