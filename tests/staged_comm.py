"""Host-staged gloo communicator: a test double of TorchComm for running
the multi-rank orchestration with several processes on ONE GPU (RCCL refuses
two ranks on one device).  Device buffers go device -> host -> gloo -> device;
the layouts (packed all-gather, rank-order all-to-all, ring halo) are
TorchComm's."""
import ctypes

import numpy as np


class HostStagedComm:
    def __init__(self, tgt):
        import torch.distributed as dist
        import hpx_amd as hpx
        self.dist = dist
        self.tgt = tgt
        self.rank, self.size = dist.get_rank(), dist.get_world_size()
        self._send = hpx.vector(8, dtype=np.int64, tgt=tgt)
        self._recv = hpx.vector(8 * self.size, dtype=np.int64, tgt=tgt)

    def _d2h(self, addr, nbytes):
        from hpx_amd import _lib as L
        buf = np.empty(nbytes, np.uint8)
        L.call("hpxhip_memcpy_async", buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(addr), nbytes, L.D2H,
               self.tgt.stream)
        self.tgt.synchronize()
        return buf

    def _h2d(self, addr, buf):
        from hpx_amd import _lib as L
        L.call("hpxhip_memcpy_async", ctypes.c_void_p(addr), buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes, L.H2D,
               self.tgt.stream)
        self.tgt.synchronize()

    def _allgather_bytes(self, b):
        import torch
        t = torch.from_numpy(b.copy())
        out = [torch.zeros_like(t) for _ in range(self.size)]
        self.dist.all_gather(out, t)
        return [o.numpy() for o in out]

    # reduce / scan / copy_if exchange
    def slots(self, nbytes):
        import hpx_amd as hpx
        words = max(1, -(-int(nbytes) // 8))
        if self._send.size() < words:
            self._send = hpx.vector(words, dtype=np.int64, tgt=self.tgt)
            self._recv = hpx.vector(words * self.size, dtype=np.int64, tgt=self.tgt)
        return self._send.data(), self._recv.data()

    def allgather(self, nbytes, stream):
        self.tgt.synchronize()
        parts = self._allgather_bytes(self._d2h(self._send.data(), nbytes))   # packed, as TorchComm
        self._h2d(self._recv.data(), np.concatenate(parts))

    def allgather_host(self, words):
        return np.stack(self._allgather_bytes(np.ascontiguousarray(words, np.int64).view(np.uint8))).view(np.int64)

    def allreduce_host(self, words):
        import torch
        t = torch.from_numpy(np.ascontiguousarray(words, np.int64).copy())
        self.dist.all_reduce(t)
        return t.numpy()

    def alltoallv(self, send_buf, send_off, send_counts, recv_buf, recv_counts, itemsize, stream, recv_off=0):
        import torch
        self.tgt.synchronize()
        n = int(sum(send_counts))
        src = torch.from_numpy(self._d2h(send_buf.data() + send_off * itemsize, n * itemsize) if n else
                               np.zeros(0, np.uint8))
        dst = torch.zeros(int(sum(recv_counts)) * itemsize, dtype=torch.uint8)
        self.dist.all_to_all_single(dst, src, [int(c) * itemsize for c in recv_counts],
                                    [int(c) * itemsize for c in send_counts])
        if dst.numel():
            self._h2d(recv_buf.data() + recv_off * itemsize, dst.numpy())

    def halo_exchange(self, send_left, send_right, recv_left, recv_right, stream, count=1):
        from hpx_amd import _lib as L
        nb = 8 * int(count)
        L.call("hpxhip_stream_synchronize", stream)
        mine = np.concatenate([self._d2h(send_left, nb), self._d2h(send_right, nb)])
        got = self._allgather_bytes(mine)
        left, right = (self.rank - 1) % self.size, (self.rank + 1) % self.size
        self._h2d(recv_left, got[left][nb:2 * nb].copy())
        self._h2d(recv_right, got[right][0:nb].copy())

    def barrier(self):
        self.dist.barrier()
