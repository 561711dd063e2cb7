"""One-shot git sync, driven by the ``GIT_SYNC_*`` environment of the
``git-sync-code`` init container (what the ``kubedl/git-sync`` image does).

Clones ``GIT_SYNC_REPO`` into ``$GIT_SYNC_ROOT/$GIT_SYNC_DEST`` (root path is
resolved inside the pod sandbox by the runtime), optionally at
``GIT_SYNC_BRANCH`` / ``GIT_SYNC_REV`` with ``--depth GIT_SYNC_DEPTH``,
retrying up to ``GIT_SYNC_MAX_SYNC_FAILURES`` times.  Credentials from
``GIT_SYNC_USERNAME``/``GIT_SYNC_PASSWORD`` are injected into an https URL;
``GIT_SYNC_SSH`` + ``GIT_SSH_KEY_FILE`` select ssh.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import time
import urllib.parse


def _url(repo: str) -> str:
    user = os.environ.get("GIT_SYNC_USERNAME")
    pw = os.environ.get("GIT_SYNC_PASSWORD")
    if user and repo.startswith(("http://", "https://")):
        u = urllib.parse.urlsplit(repo)
        netloc = f"{urllib.parse.quote(user)}:{urllib.parse.quote(pw or '')}@{u.hostname}"
        if u.port:
            netloc += f":{u.port}"
        return urllib.parse.urlunsplit((u.scheme, netloc, u.path, u.query, u.fragment))
    return repo


def sync_once(env=os.environ) -> str:
    repo = env["GIT_SYNC_REPO"]
    root = env.get("GIT_SYNC_ROOT", "/code")
    dest = env.get("GIT_SYNC_DEST") or os.path.basename(repo.rstrip("/")).removesuffix(".git")
    target = os.path.join(root, dest)
    tmp = target + ".tmp-sync"
    shutil.rmtree(tmp, ignore_errors=True)
    os.makedirs(root, exist_ok=True)
    cmd = ["git", "clone", "--quiet"]
    if env.get("GIT_SYNC_DEPTH"):
        cmd += ["--depth", env["GIT_SYNC_DEPTH"]]
    if env.get("GIT_SYNC_BRANCH"):
        cmd += ["--branch", env["GIT_SYNC_BRANCH"]]
    cmd += [_url(repo), tmp]
    genv = dict(env)
    if env.get("GIT_SYNC_SSH") == "true" and env.get("GIT_SSH_KEY_FILE"):
        genv["GIT_SSH_COMMAND"] = f"ssh -i {env['GIT_SSH_KEY_FILE']} -o StrictHostKeyChecking=no"
    subprocess.run(cmd, check=True, env=genv)
    if env.get("GIT_SYNC_REV"):
        subprocess.run(["git", "-C", tmp, "checkout", "--quiet", env["GIT_SYNC_REV"]], check=True, env=genv)
    shutil.rmtree(target, ignore_errors=True)
    os.replace(tmp, target)
    return target


def main() -> int:
    tries = max(1, int(os.environ.get("GIT_SYNC_MAX_SYNC_FAILURES", "3") or 3))
    for i in range(tries):
        try:
            path = sync_once()
            print(f"git-sync: synced into {path}", flush=True)
            return 0
        except (subprocess.CalledProcessError, OSError, KeyError) as e:
            print(f"git-sync: attempt {i + 1}/{tries} failed: {e}", file=sys.stderr, flush=True)
            time.sleep(min(2 ** i, 10) * 0.1)
    return 1


if __name__ == "__main__":
    sys.exit(main())
