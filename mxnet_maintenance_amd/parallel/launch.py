"""Local multi-process launcher: one worker process per MI355X.

Parity: the reference's ``tools/launch.py:57`` (``--launcher local``) starts
``-n`` worker processes (and ps-lite servers/scheduler) with the DMLC_* role
environment.  Here there is no parameter server: every worker is a peer in one
``torch.distributed`` process group (RCCL over xGMI for GPU tensors, gloo on
CPU), so launching means starting N fresh child processes with
RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT
set and waiting for all of them.

The launcher itself never touches the GPU (no HIP call, not even
``torch.cuda.is_available()``): on this platform a process that has
initialised HIP must not fork/exec GPU children, and the parent of a job is the
natural place for such mistakes.  If any worker fails, the remaining ones are
terminated and the first failing exit code is returned.
"""
import os
import signal
import socket
import subprocess
import sys
import time

__all__ = ['free_port', 'worker_env', 'launch', 'relaunch_self']


def free_port(host='127.0.0.1'):
    """An unused TCP port on ``host`` (for MASTER_PORT)."""
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    try:
        s.bind((host, 0))
        return s.getsockname()[1]
    finally:
        s.close()


def worker_env(rank, nproc, master_addr='127.0.0.1', master_port=None, base=None, extra=None):
    """Environment of worker ``rank`` of a single-node job of ``nproc`` workers."""
    env = dict(os.environ if base is None else base)
    env.update({
        'RANK': str(rank), 'LOCAL_RANK': str(rank), 'WORLD_SIZE': str(nproc),
        'LOCAL_WORLD_SIZE': str(nproc), 'GROUP_RANK': '0',
        'MASTER_ADDR': master_addr, 'MASTER_PORT': str(master_port or 29500),
    })
    # dmabuf IPC is the only mode the host driver supports; RCCL/IPC fail without it
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    env.setdefault('OMP_NUM_THREADS', '1' if nproc > 1 else env.get('OMP_NUM_THREADS', '1'))
    if extra:
        env.update({k: str(v) for k, v in extra.items()})
    return env


def launch(cmd, nproc, master_addr='127.0.0.1', master_port=None, extra_env=None, timeout=None, poll_s=0.2):
    """Run ``cmd`` (argv list) as ``nproc`` local workers; return the job's exit code.

    Exit code: 0 if every worker exited 0, else the first non-zero code observed
    (the other workers are then terminated, so a crashed rank cannot leave its
    peers blocked in a collective until the process-group timeout).
    """
    if nproc < 1:
        raise ValueError('nproc must be >= 1')
    port = master_port or free_port(master_addr)
    procs = []
    for r in range(nproc):
        env = worker_env(r, nproc, master_addr, port, extra=extra_env)
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
    t0 = time.time()
    code = 0
    try:
        while True:
            alive = 0
            for p in procs:
                rc = p.poll()
                if rc is None:
                    alive += 1
                elif rc != 0 and code == 0:
                    code = rc
            if code != 0 or alive == 0:
                break
            if timeout is not None and time.time() - t0 > timeout:
                code = 124
                break
            time.sleep(poll_s)
    except KeyboardInterrupt:
        code = 130
    finally:
        if code != 0:
            _terminate(procs)
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                _kill_group(p, signal.SIGKILL)
                p.wait()
    if code < 0:          # killed by a signal: shell convention
        code = 128 - code
    return code


def _kill_group(p, sig):
    try:
        os.killpg(p.pid, sig)
    except (ProcessLookupError, PermissionError):
        pass


def _terminate(procs):
    for p in procs:
        if p.poll() is None:
            _kill_group(p, signal.SIGTERM)
    deadline = time.time() + 15
    for p in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.1)
        if p.poll() is None:
            _kill_group(p, signal.SIGKILL)


def relaunch_self(nproc, argv=None, script=None, extra_env=None):
    """Start ``nproc`` copies of the running script as workers and return the exit code.

    Used by entry points (``bench.py --gpus N``) when they are started without
    a launcher: call it BEFORE anything initialises the GPU.
    """
    argv = list(sys.argv[1:] if argv is None else argv)
    script = script or os.path.abspath(sys.argv[0])
    return launch([sys.executable, '-u', script] + argv, nproc, extra_env=extra_env)


def needs_launch(requested):
    """True when ``requested`` workers were asked for but this process is not one of a job."""
    return requested > 1 and 'WORLD_SIZE' not in os.environ and 'RANK' not in os.environ
