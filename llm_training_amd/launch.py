"""In-process multi-rank launcher: one child process per GPU, started by the command itself.

Reference behaviour: Lightning's ``_SubprocessScriptLauncher`` — ``llm-training fit`` with N devices
re-executes itself N times, one process per GPU (src/llm_training/lightning/strategy/fsdp2/
fsdp2_strategy.py:169-173) — and the SLURM template's ``srun`` launch (scripts/train.sh:17-35).

Here the parent stays a plain supervisor:

* It makes **no HIP call at all** (no ``torch.cuda.*``, not even ``device_count()``): a GPU count for
  ``devices: auto`` comes from a short-lived probe child. The children are fresh interpreters
  (``subprocess``, never fork/exec of a process that touched the GPU), each pinned to its GPU through
  ``LOCAL_RANK`` and rendezvousing over TCP on 127.0.0.1 (``MASTER_ADDR`` / a free ``MASTER_PORT``).
* The RCCL environment every rank needs on MI355X hosts is set in the children's environment
  (``HSA_ENABLE_IPC_MODE_LEGACY=0``: the host driver only supports dmabuf IPC, so RCCL's P2P buffers
  over xGMI fail without it). ``apply_rccl_env()`` sets the same defaults for torchrun / srun users.
* It waits for all ranks. The first child that exits non-zero ends the job: the others (each in its
  own process group) get SIGTERM, then SIGKILL after a grace period, and the parent returns that exit
  code — a crashed rank never leaves the rest blocked in a collective until the 30-minute timeout.
* Output is not captured: every child writes to the parent's stdout / stderr, so rank 0's JSON
  line (bench.py) or log reaches the caller unchanged.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time

# Defaults every GPU rank needs (setdefault: an explicit user value wins).
RCCL_ENV = {
    # dmabuf IPC: legacy IPC handles are rejected by the MI355X host driver (hipIpcGetMemHandle fails)
    "HSA_ENABLE_IPC_MODE_LEGACY": "0",
}

LAUNCHED_ENV = "LLMT_LAUNCHED"  # set in children: never launch again from inside a rank


def apply_rccl_env(env: dict | None = None) -> dict:
    """setdefault the RCCL environment into ``env`` (``os.environ`` by default); returns it."""
    env = os.environ if env is None else env
    for k, v in RCCL_ENV.items():
        env.setdefault(k, v)
    return env


def externally_launched() -> bool:
    """True inside a rank started by torchrun / srun / this launcher."""
    if os.environ.get(LAUNCHED_ENV) == "1":
        return True
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        return True
    return "SLURM_PROCID" in os.environ and int(os.environ.get("SLURM_NTASKS", "1")) > 1


def env_world_size() -> int | None:
    if "WORLD_SIZE" in os.environ:
        return int(os.environ["WORLD_SIZE"])
    if "SLURM_PROCID" in os.environ and int(os.environ.get("SLURM_NTASKS", "1")) > 1:
        return int(os.environ["SLURM_NTASKS"])
    return None


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def probe_gpu_count(timeout: float = 300.0) -> int:
    """Number of visible GPUs, counted in a throw-away child so this process never initialises HIP."""
    code = "import torch; print(torch.cuda.device_count() if torch.cuda.is_available() else 0)"
    try:
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout,
                           env=apply_rccl_env(dict(os.environ)))
        return int(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 and r.stdout.strip() else 0
    except (subprocess.TimeoutExpired, ValueError, IndexError):
        return 0


def resolve_devices(devices, accelerator="auto") -> int:
    """Lightning ``trainer.devices`` → number of processes on this node (int, "auto", "-1", list)."""
    if accelerator == "cpu":
        return max(1, int(devices)) if isinstance(devices, int) or str(devices).isdigit() else 1
    if devices is None or devices == "auto" or str(devices) == "-1" or devices == -1:
        n = probe_gpu_count() if os.path.exists("/dev/kfd") else 0  # no ROCm device node: CPU host
        return max(1, n)
    if isinstance(devices, (list, tuple)):
        return len(devices)
    if isinstance(devices, str) and "," in devices:
        return len([d for d in devices.split(",") if d.strip()])
    return max(1, int(devices))


def device_list(devices) -> list[int] | None:
    """The explicit GPU indices of ``trainer.devices`` (a list or "2,3"), or None for a count / auto."""
    if isinstance(devices, (list, tuple)):
        return [int(d) for d in devices]
    if isinstance(devices, str) and "," in devices:
        return [int(d) for d in devices.split(",") if d.strip()]
    return None


def visible_devices_env(ids: list[int], env: dict | None = None) -> dict:
    """HIP_VISIBLE_DEVICES (and CUDA_VISIBLE_DEVICES, its alias, set to the same list so that no stale
    parent value disagrees with it whichever one the runtime reads) for ranks pinned to the listed GPUs
    (Lightning semantics: indices into the GPUs this process sees). Every child sees exactly the listed
    GPUs, in order, so LOCAL_RANK r runs on ``ids[r]``; an existing HIP_VISIBLE_DEVICES (else
    CUDA_VISIBLE_DEVICES) selection is composed with it. ROCR_VISIBLE_DEVICES is applied by the ROCm
    runtime below HIP (HIP's indices count within it), so it is passed through unchanged."""
    env = os.environ if env is None else env
    base = env.get("HIP_VISIBLE_DEVICES") or env.get("CUDA_VISIBLE_DEVICES")
    if base:
        vis = [x.strip() for x in base.split(",") if x.strip()]
        if max(ids) >= len(vis):
            raise SystemExit(f"trainer.devices {ids}: only {len(vis)} GPUs are visible ({base})")
        sel = [vis[i] for i in ids]
    else:
        sel = [str(i) for i in ids]
    if len(set(sel)) != len(sel):
        raise SystemExit(f"trainer.devices {ids} lists a GPU twice")
    return {"HIP_VISIBLE_DEVICES": ",".join(sel), "CUDA_VISIBLE_DEVICES": ",".join(sel)}


def _kill_group(p: subprocess.Popen, sig) -> None:
    try:
        os.killpg(p.pid, sig)
    except (ProcessLookupError, PermissionError):
        pass


def spawn(nprocs: int, cmd: list[str], *, env: dict | None = None, grace: float = 10.0,
          poll: float = 0.2, master_port: int | None = None, extra_env: dict | None = None) -> int:
    """Run ``cmd`` as ``nprocs`` ranks on this node and supervise them; returns the job's exit code
    (0 when every rank succeeded, else the first failing rank's code; -N for a signal maps to 128+N)."""
    base = apply_rccl_env(dict(os.environ if env is None else env))
    # the children import this package from the same tree as the parent (in-tree _C.so included)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pp = base.get("PYTHONPATH", "")
    if root not in pp.split(os.pathsep):
        base["PYTHONPATH"] = root + (os.pathsep + pp if pp else "")
    port = master_port or free_port()
    procs: list[subprocess.Popen] = []
    try:
        for r in range(nprocs):
            e = dict(base)
            e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(nprocs),
                      "LOCAL_WORLD_SIZE": str(nprocs), "GROUP_RANK": "0", "NODE_RANK": "0",
                      "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), LAUNCHED_ENV: "1"})
            for k in ("SLURM_PROCID", "SLURM_NTASKS", "SLURM_LOCALID"):  # this launcher owns the ranks
                e.pop(k, None)
            if extra_env:
                e.update(extra_env)
            procs.append(subprocess.Popen(cmd, env=e, start_new_session=True))
        failed: tuple[int, int] | None = None
        while True:
            alive = 0
            for r, p in enumerate(procs):
                rc = p.poll()
                if rc is None:
                    alive += 1
                elif rc != 0 and failed is None:
                    failed = (r, rc)
            if failed is not None or alive == 0:
                break
            time.sleep(poll)
        if failed is not None:
            r, rc = failed
            print(f"[launch] rank {r} exited with {rc}; stopping the other ranks", file=sys.stderr, flush=True)
            _terminate(procs, grace)
            return rc if rc > 0 else 128 + (-rc)
        return 0
    except KeyboardInterrupt:
        _terminate(procs, grace)
        return 130
    finally:
        _terminate(procs, grace)


def _terminate(procs: list[subprocess.Popen], grace: float) -> None:
    live = [p for p in procs if p.poll() is None]
    if not live:
        return
    for p in live:
        _kill_group(p, signal.SIGTERM)
    deadline = time.time() + grace
    for p in live:
        try:
            p.wait(timeout=max(0.0, deadline - time.time()))
        except subprocess.TimeoutExpired:
            pass
    for p in live:
        if p.poll() is None:
            _kill_group(p, signal.SIGKILL)
            p.wait()


def launch_for_trainer(trainer_cfg: dict, cmd: list[str]) -> int | None:
    """``llm-training fit``: spawn ``trainer.devices`` ranks on this node (Lightning semantics) unless a
    launcher already did. Multi-node jobs (``num_nodes`` > 1) must come from srun / torchrun."""
    devices = trainer_cfg.get("devices", "auto")
    accelerator = trainer_cfg.get("accelerator", "auto")
    num_nodes = int(trainer_cfg.get("num_nodes", 1) or 1)
    if externally_launched():
        ws = env_world_size()
        explicit = isinstance(devices, (int, list, tuple)) or (isinstance(devices, str) and devices.isdigit())
        if explicit and ws is not None:
            want = resolve_devices(devices, accelerator) * num_nodes
            if want != ws:
                raise SystemExit(f"trainer.devices x num_nodes = {want} but the launcher started WORLD_SIZE={ws}")
        apply_rccl_env()
        return None
    if num_nodes > 1:
        raise SystemExit("trainer.num_nodes > 1 needs one task per GPU from srun or torchrun "
                         "(see scripts/train.sh)")
    ids = device_list(devices) if accelerator != "cpu" else None
    if ids is not None and ids != list(range(len(ids))):
        # GPUs other than the first n: every rank sees exactly the listed ones (a single rank too)
        extra = visible_devices_env(ids)
        if len(ids) == 1:
            os.environ.update(extra)  # this process becomes the rank: no HIP call has happened yet
            apply_rccl_env()
            return None
        apply_rccl_env()
        return spawn(len(ids), cmd, extra_env=extra)
    return maybe_launch(resolve_devices(devices, accelerator), cmd)


def maybe_launch(nprocs: int, cmd: list[str]) -> int | None:
    """Launch ``cmd`` as ``nprocs`` ranks unless already inside a rank. Returns the exit code of the
    job when it launched, None when the caller should run in this process (nprocs == 1, or torchrun /
    srun / this launcher already started it — then WORLD_SIZE must equal nprocs)."""
    if externally_launched():
        ws = env_world_size()
        if ws is not None and ws != nprocs:
            raise SystemExit(f"requested {nprocs} processes in total but the launcher started WORLD_SIZE={ws}")
        apply_rccl_env()
        return None
    apply_rccl_env()
    if nprocs <= 1:
        return None
    return spawn(nprocs, cmd)
