"""Stand-in for the SimPy 4 core, used ONLY to run the reference in this container.

TEST INFRASTRUCTURE. The reference (`/root/reference`, requirements.txt:6 `simpy>=4.0.0`)
depends on SimPy, which is not installed and cannot be fetched offline.  This module
restates the published SimPy 4 core semantics that the reference exercises:

* ``Environment``: heap of ``(time, priority, eid, event)``; ``step()`` pops the head,
  sets ``now``, detaches ``callbacks`` and calls each one, then re-raises the value of a
  failed, un-defused event; ``run(until=t)`` schedules a pre-succeeded stop event with
  URGENT priority at ``float(t)``.
* ``Event.succeed`` schedules NORMAL at delay 0; ``Timeout(d)`` schedules NORMAL at d;
  ``Initialize`` schedules URGENT at delay 0 with ``callbacks=[proc._resume]``.
* ``Process._resume`` drives the generator; an already-processed yielded event is
  resumed immediately, otherwise ``_resume`` is appended to its callbacks.  On
  ``StopIteration`` / exception the process schedules itself (NORMAL) ok / failed.
* ``Resource(capacity)``: ``users``, ``put_queue``, ``get_queue``; ``Request`` appends to
  ``put_queue``, registers ``_trigger_get`` as its callback and calls ``_trigger_put``,
  which only inspects the head of the put queue (``_do_put`` returns None).
  ``Request.__exit__`` cancels an untriggered request and then releases;
  ``Release`` appends to ``get_queue``, registers ``_trigger_put`` and calls
  ``_trigger_get`` (``_do_get`` removes the user and succeeds).

Call sites in the reference: FJSPSimulation.py:45,183-184,302; agents/AGVAgent.py:236,393;
agents/MachineAgent.py:50,121,156-165; agents/PackagingAgent.py:46,115,135-141,151.
Parity with the real SimPy package is therefore *unpinned* (no SimPy in this image);
these rules are the spec.
"""
from heapq import heappush, heappop
from itertools import count

URGENT = 0
NORMAL = 1
PENDING = object()


class StopSimulation(Exception):
    @classmethod
    def callback(cls, event):
        if event._ok:
            raise cls(event._value)
        raise event._value


class EmptySchedule(Exception):
    pass


class Event:
    def __init__(self, env):
        self.env = env
        self.callbacks = []
        self._value = PENDING

    @property
    def triggered(self):
        return self._value is not PENDING

    @property
    def processed(self):
        return self.callbacks is None

    @property
    def ok(self):
        return self._ok

    @property
    def value(self):
        if self._value is PENDING:
            raise AttributeError("value of %s is not yet available" % self)
        return self._value

    def succeed(self, value=None):
        if self._value is not PENDING:
            raise RuntimeError("%s has already been triggered" % self)
        self._ok = True
        self._value = value
        self.env.schedule(self)
        return self

    def fail(self, exception):
        if self._value is not PENDING:
            raise RuntimeError("%s has already been triggered" % self)
        self._ok = False
        self._value = exception
        self.env.schedule(self)
        return self


class Timeout(Event):
    def __init__(self, env, delay, value=None):
        if delay < 0:
            raise ValueError("Negative delay %s" % delay)
        self.env = env
        self.callbacks = []
        self._value = value
        self._delay = delay
        self._ok = True
        env.schedule(self, NORMAL, delay)


class Initialize(Event):
    def __init__(self, env, process):
        self.env = env
        self.callbacks = [process._resume]
        self._value = None
        self._ok = True
        env.schedule(self, URGENT)


class Process(Event):
    def __init__(self, env, generator):
        if not hasattr(generator, "throw"):
            raise ValueError("%s is not a generator." % generator)
        self.env = env
        self.callbacks = []
        self._value = PENDING
        self._generator = generator
        self._target = Initialize(env, self)

    @property
    def is_alive(self):
        return self._value is PENDING

    def _resume(self, event):
        self.env._active_proc = self
        while True:
            try:
                if event._ok:
                    event = self._generator.send(event._value)
                else:
                    event._defused = True
                    exc = type(event._value)(*event._value.args)
                    exc.__cause__ = event._value
                    event = self._generator.throw(exc)
            except StopIteration as e:
                event = None
                self._ok = True
                self._value = e.args[0] if len(e.args) else None
                self.env.schedule(self)
                break
            except BaseException as e:
                event = None
                self._ok = False
                self._value = e
                self.env.schedule(self)
                break
            if event.callbacks is not None:
                event.callbacks.append(self._resume)
                break
        self._target = event
        self.env._active_proc = None


class Environment:
    def __init__(self, initial_time=0):
        self._now = initial_time
        self._queue = []
        self._eid = count()
        self._active_proc = None

    @property
    def now(self):
        return self._now

    @property
    def active_process(self):
        return self._active_proc

    def process(self, generator):
        return Process(self, generator)

    def timeout(self, delay, value=None):
        return Timeout(self, delay, value)

    def event(self):
        return Event(self)

    def schedule(self, event, priority=NORMAL, delay=0):
        heappush(self._queue, (self._now + delay, priority, next(self._eid), event))

    def peek(self):
        try:
            return self._queue[0][0]
        except IndexError:
            return float("inf")

    def step(self):
        try:
            self._now, _, _, event = heappop(self._queue)
        except IndexError:
            raise EmptySchedule()
        callbacks, event.callbacks = event.callbacks, None
        for callback in callbacks:
            callback(event)
        if not event._ok and not hasattr(event, "_defused"):
            exc = type(event._value)(*event._value.args)
            exc.__cause__ = event._value
            raise exc

    def run(self, until=None):
        if until is not None:
            if not isinstance(until, Event):
                at = float(until)
                if at <= self.now:
                    raise ValueError("until(=%s) must be > the current simulation time." % at)
                until = Event(self)
                until._ok = True
                until._value = None
                self.schedule(until, URGENT, at - self.now)
            elif until.callbacks is None:
                return until.value
            until.callbacks.append(StopSimulation.callback)
        try:
            while True:
                self.step()
        except StopSimulation as exc:
            return exc.args[0]
        except EmptySchedule:
            if until is not None:
                raise RuntimeError("No scheduled events left but until event was not triggered")
        return None


class Put(Event):
    def __init__(self, resource):
        super().__init__(resource._env)
        self.resource = resource
        self.proc = self.env.active_process
        resource.put_queue.append(self)
        self.callbacks.append(resource._trigger_get)
        resource._trigger_put(None)

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc_value, traceback):
        self.cancel()
        return None

    def cancel(self):
        if not self.triggered:
            self.resource.put_queue.remove(self)


class Get(Event):
    def __init__(self, resource):
        super().__init__(resource._env)
        self.resource = resource
        self.proc = self.env.active_process
        resource.get_queue.append(self)
        self.callbacks.append(resource._trigger_put)
        resource._trigger_get(None)

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc_value, traceback):
        self.cancel()
        return None

    def cancel(self):
        if not self.triggered:
            self.resource.get_queue.remove(self)


class Request(Put):
    def __exit__(self, exc_type, exc_value, traceback):
        super().__exit__(exc_type, exc_value, traceback)
        if exc_type is not GeneratorExit:
            self.resource.release(self)
        return None


class Release(Get):
    def __init__(self, resource, request):
        self.request = request
        super().__init__(resource)


class Resource:
    def __init__(self, env, capacity=1):
        if capacity <= 0:
            raise ValueError('"capacity" must be > 0.')
        self._env = env
        self._capacity = capacity
        self.put_queue = []
        self.get_queue = []
        self.users = []
        self.queue = self.put_queue

    @property
    def capacity(self):
        return self._capacity

    @property
    def count(self):
        return len(self.users)

    def request(self):
        return Request(self)

    def release(self, request):
        return Release(self, request)

    def _do_put(self, event):
        if len(self.users) < self.capacity:
            self.users.append(event)
            event.usage_since = self._env.now
            event.succeed()

    def _do_get(self, event):
        try:
            self.users.remove(event.request)
        except ValueError:
            pass
        event.succeed()

    def _trigger_put(self, get_event):
        idx = 0
        while idx < len(self.put_queue):
            put_event = self.put_queue[idx]
            proceed = self._do_put(put_event)
            if not put_event.triggered:
                idx += 1
            elif self.put_queue.pop(idx) != put_event:
                raise RuntimeError("Put queue invariant violated")
            if not proceed:
                break

    def _trigger_get(self, put_event):
        idx = 0
        while idx < len(self.get_queue):
            get_event = self.get_queue[idx]
            proceed = self._do_get(get_event)
            if not get_event.triggered:
                idx += 1
            elif self.get_queue.pop(idx) != get_event:
                raise RuntimeError("Get queue invariant violated")
            if not proceed:
                break
