"""Execution policies: seq, par, par_unseq, task, .on(executor), .with_(params).

Mirrors hpx/parallel/execution_policy.hpp: ``sequenced_policy`` (seq, 478),
``parallel_policy`` (par, 1054), ``parallel_unsequenced_policy``, the task
variants (``par(task)``, 639), rebinding with ``.on(exec)`` (980-998) and
``.with(params)`` (1014-1026; ``with`` is a Python keyword, hence
``with_``).  Executor parameters such as ``static_chunk_size`` are accepted
and carried for API parity; the GPU kernels choose their own tiling.
"""
from __future__ import annotations

from dataclasses import dataclass, replace


class _task_tag:
    def __repr__(self):
        return "hpx::parallel::execution::task"


task = _task_tag()


@dataclass(frozen=True)
class static_chunk_size:
    """execution parameters (static_chunk_size.hpp:54-69)."""
    chunk_size: int = 0


@dataclass(frozen=True)
class auto_chunk_size:
    pass


@dataclass(frozen=True)
class dynamic_chunk_size:
    chunk_size: int = 1


@dataclass(frozen=True)
class policy:
    name: str
    is_task: bool = False
    executor: object = None
    parameters: object = None
    sequenced: bool = False

    def __call__(self, tag):
        if tag is not task:
            raise TypeError("policy(task) expects hpx::parallel::execution::task")
        return replace(self, is_task=True, name=self.name + "(task)")

    def on(self, executor):
        return replace(self, executor=executor)

    def with_(self, *params):
        return replace(self, parameters=params[0] if len(params) == 1 else params)

    def executor_or_none(self):
        return self.executor

    def __repr__(self):
        s = self.name
        if self.executor is not None:
            s += f".on({type(self.executor).__name__})"
        return s


seq = policy("seq", sequenced=True)
par = policy("par")
par_unseq = policy("par_unseq")
unseq = policy("unseq")
sequenced_policy = seq
parallel_policy = par


def is_execution_policy(p) -> bool:
    return isinstance(p, policy)


def is_async_execution_policy(p) -> bool:
    return isinstance(p, policy) and p.is_task
