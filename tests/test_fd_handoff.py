"""The cross-process device ring's fd hand-off (shmring.hpp FdHandoff /
shm_receive_fd), on the CPU: a memfd stands in for the GPU ring's dma-buf.  A
separate process receives the fd over the abstract unix socket, maps it and
writes through the mapping; the owner sees the write in its own mapping -- the
same steps a client process takes to publish into a server GPU's request ring
(test_shm_rpc_gpu.py runs them against the real dma-buf)."""
import mmap
import os

import pytest
import torch.multiprocessing as mp

from ptype_amd import _core


def _peer(name, q):
    from ptype_amd import _core as C

    fd = C.fd_receive(name)
    m = mmap.mmap(fd, 4096, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
    os.close(fd)
    seen = bytes(m[:5])
    m[64:69] = b"reply"
    m.close()
    q.put(seen)


def test_fd_handoff_maps_the_same_memory_in_another_process():
    fd = os.memfd_create("ptype-test-ring")
    os.ftruncate(fd, 4096)
    mine = mmap.mmap(fd, 4096, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
    mine[:5] = b"hello"
    name = f"ptype-test-handoff-{os.getpid()}"
    h = _core.FdHandoff(name, fd)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_peer, args=(name, q))
    p.start()
    assert q.get(timeout=60) == b"hello"
    p.join(30)
    assert p.exitcode == 0
    assert bytes(mine[64:69]) == b"reply"
    assert h.handed == 1
    del h
    mine.close()
    os.close(fd)


def test_fd_receive_fails_cleanly_without_a_server():
    with pytest.raises(Exception, match="fd hand-off"):
        _core.fd_receive(f"ptype-test-nobody-{os.getpid()}")
