"""The `dpe` command line's RCCL-id rendezvous (dpe-mvs_amd/host/rdzv.h), driven on the CPU: rank 0
answers only connections whose hello carries a valid rank and this run's token, so intruders (a
port probe, a wrong-token peer, a duplicate rank) neither use up a slot nor receive the id."""
import os
import socket
import struct
import subprocess
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("rdzv") / "rdzv_driver")
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", exe, os.path.join(ROOT, "tests", "rdzv_driver.cpp"), "-lpthread"],
                   check=True)
    return exe


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env(port, run_id="job-a"):
    e = dict(os.environ)
    e.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port - 1), TORCHELASTIC_RUN_ID=run_id)
    e.pop("DPE_RDZV_PORT", None)
    return e


def _connect(port, timeout=10.0):
    t0 = time.time()
    while True:
        try:
            return socket.create_connection(("127.0.0.1", port), timeout=2)
        except OSError:
            if time.time() - t0 > timeout:
                raise
            time.sleep(0.05)


EXPECTED = "".join(f"{(i * 37 + 11) & 255:02x}" for i in range(128))


def test_ranks_get_the_id_despite_intruders(driver):
    port = _free_port()
    world = 3
    r0 = subprocess.Popen([driver, "0", str(world)], env=_env(port), stdout=subprocess.PIPE, text=True)
    # intruders first: a probe that closes at once, a wrong-token hello, an out-of-range rank
    s = _connect(port)
    s.close()
    for rank, token in ((1, 12345), (7, None)):
        s = _connect(port)
        if token is None:   # right token shape is unknown to an intruder: send garbage of hello size
            s.sendall(struct.pack("<IiQ", 0x44504531, rank, 0))
        else:
            s.sendall(struct.pack("<IiQ", 0x44504531, rank, token))
        s.settimeout(5)
        assert s.recv(128) == b"", "an intruder received the id"
        s.close()
    outs = [subprocess.run([driver, str(r), str(world)], env=_env(port), capture_output=True, text=True, timeout=60)
            for r in (1, 2)]
    r0_out, _ = r0.communicate(timeout=60)
    assert r0.returncode == 0 and r0_out.strip() == EXPECTED
    for o in outs:
        assert o.returncode == 0 and o.stdout.strip() == EXPECTED


def test_other_job_cannot_take_a_slot(driver):
    port = _free_port()
    r0 = subprocess.Popen([driver, "0", "2"], env=_env(port, "job-a"), stdout=subprocess.PIPE, text=True)
    time.sleep(0.2)
    other = subprocess.Popen([driver, "1", "2"], env=_env(port, "job-b"), stdout=subprocess.PIPE, text=True)
    time.sleep(1.0)
    assert r0.poll() is None, "rank 0 finished with a peer from another job"
    mine = subprocess.run([driver, "1", "2"], env=_env(port, "job-a"), capture_output=True, text=True, timeout=60)
    r0_out, _ = r0.communicate(timeout=60)
    assert mine.stdout.strip() == EXPECTED and r0_out.strip() == EXPECTED
    other.kill()
    other.wait()


def test_silent_connections_do_not_starve_the_ranks(driver):
    # connections that never send a hello are served concurrently with a 2 s budget each, so the
    # real ranks get the id at once instead of after 5 s per silent peer
    port = _free_port()
    r0 = subprocess.Popen([driver, "0", "3"], env=_env(port), stdout=subprocess.PIPE, text=True)
    silent = [_connect(port) for _ in range(12)]
    t0 = time.time()
    outs = [subprocess.Popen([driver, str(r), "3"], env=_env(port), stdout=subprocess.PIPE, text=True) for r in (1, 2)]
    res = [o.communicate(timeout=60)[0].strip() for o in outs]
    r0_out, _ = r0.communicate(timeout=60)
    took = time.time() - t0
    for s in silent:
        s.close()
    assert res == [EXPECTED, EXPECTED] and r0_out.strip() == EXPECTED
    assert took < 6.0, took


def test_shared_secret_authenticates(driver):
    # with DPE_RDZV_SECRET set on the job's ranks, a peer that knows the run id but not the secret
    # gets nothing and takes no slot
    port = _free_port()
    env = _env(port)
    env["DPE_RDZV_SECRET"] = "s3cr3t-nonce"
    r0 = subprocess.Popen([driver, "0", "2"], env=env, stdout=subprocess.PIPE, text=True)
    time.sleep(0.2)
    nosecret = subprocess.Popen([driver, "1", "2"], env=_env(port), stdout=subprocess.PIPE, text=True)
    time.sleep(1.0)
    assert r0.poll() is None, "rank 0 served a peer without the secret"
    mine = subprocess.run([driver, "1", "2"], env=env, capture_output=True, text=True, timeout=60)
    r0_out, _ = r0.communicate(timeout=60)
    assert mine.stdout.strip() == EXPECTED and r0_out.strip() == EXPECTED
    nosecret.kill()
    nosecret.wait()


@pytest.mark.parametrize("addr,resolved,lws,secret,expect", [
    ("127.0.0.1", "127.0.0.1", None, "s3", "127.0.0.1"),      # numeric loopback literal: never widened
    ("localhost", "127.0.0.1", None, "s3", "127.0.0.1"),      # "localhost": never widened
    ("node7", "127.0.1.1", None, None, "127.0.1.1"),          # hostname -> loopback, no secret: kept (warning)
    ("node7", "127.0.1.1", None, "s3", "0.0.0.0"),            # hostname -> loopback, secret: every interface
    ("node7", "127.0.1.1", "4", "s3", "127.0.1.1"),           # all ranks local: kept
    ("node7", "10.1.2.3", None, "s3", "10.1.2.3"),            # a routable address: itself
])
def test_listen_address(driver, addr, resolved, lws, secret, expect):
    """rank 0 widens its listener only for a host name that resolves to loopback, with ranks
    off this host and DPE_RDZV_SECRET set (the only case where the hello token authenticates)."""
    e = dict(os.environ)
    for k in ("LOCAL_WORLD_SIZE", "DPE_RDZV_SECRET"):
        e.pop(k, None)
    if lws:
        e["LOCAL_WORLD_SIZE"] = lws
    if secret:
        e["DPE_RDZV_SECRET"] = secret
    out = subprocess.run([driver, "bind", addr, resolved, "4"], env=e, capture_output=True, text=True, check=True)
    assert out.stdout.strip() == expect
    assert ("DPE_RDZV_SECRET" in out.stderr) == (addr == "node7" and resolved.startswith("127.") and not secret and not lws)
