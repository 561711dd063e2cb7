// kubedl_amd._native: the rank-process supervisor primitives of the local
// runtime (the "kubelet" that replaces Kubernetes pods with processes).
//
// Why native: a rank must be started from a multi-threaded controller
// process (watch handlers, reconcile workers, HTTP metrics) with
//   * its own session / process group (so a whole rank tree -- torchrun
//     children, RCCL proxy threads' helpers -- is signalled at once),
//   * PR_SET_PDEATHSIG so ranks die with the runtime instead of leaking GPUs,
//   * stdout/stderr redirected to the pod's log files,
//   * a reliable "exec failed" channel (errno over a CLOEXEC pipe) so a bad
//     command becomes exit code 127/126 like a container runtime reports.
// Everything between fork() and execve() is async-signal-safe: argv/envp are
// materialised before fork, the child only calls setsid/prctl/open/dup2/
// chdir/execve/write/_exit.  Python's subprocess cannot give PDEATHSIG without
// preexec_fn, which is unsafe in threaded programs.
//
// API (all return Python ints/tuples):
//   spawn(argv: list[str], env: list[str], cwd: str|None, out: str|None,
//         err: str|None, pdeathsig: int = SIGKILL) -> pid
//   reap(pids: list[int]) -> list[(pid, exit_code)]   (exit_code = status,
//         or 128 + signal, container-runtime convention); non-blocking
//   kill_group(pid, sig) -> 0 / -errno
//   alive(pid) -> bool
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <string.h>
#include <sys/prctl.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>

#include <string>
#include <vector>

namespace {

bool to_strings(PyObject* seq, std::vector<std::string>* out, const char* what) {
  PyObject* fast = PySequence_Fast(seq, what);
  if (!fast) return false;
  Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
  out->reserve(n);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* it = PySequence_Fast_GET_ITEM(fast, i);
    const char* s = PyUnicode_AsUTF8(it);
    if (!s) {
      Py_DECREF(fast);
      return false;
    }
    out->emplace_back(s);
  }
  Py_DECREF(fast);
  return true;
}

// Search PATH from the CHILD's env (execvpe semantics without malloc).
void exec_search(const char* file, char* const argv[], char* const envp[], const char* path) {
  if (strchr(file, '/')) {
    execve(file, argv, envp);
    return;
  }
  char buf[4096];
  const char* p = path && *path ? path : "/usr/local/bin:/usr/bin:/bin";
  int saved = ENOENT;
  while (*p) {
    const char* e = strchr(p, ':');
    size_t len = e ? static_cast<size_t>(e - p) : strlen(p);
    size_t flen = strlen(file);
    if (len + 1 + flen + 1 < sizeof(buf)) {
      memcpy(buf, p, len);
      size_t o = len;
      if (o == 0) buf[o++] = '.';
      buf[o++] = '/';
      memcpy(buf + o, file, flen + 1);
      execve(buf, argv, envp);
      if (errno != ENOENT && errno != ENOTDIR) saved = errno;
    }
    if (!e) break;
    p = e + 1;
  }
  errno = saved;
}

PyObject* py_spawn(PyObject*, PyObject* args, PyObject* kw) {
  static const char* kwlist[] = {"argv", "env", "cwd", "out", "err", "pdeathsig", nullptr};
  PyObject *py_argv, *py_env;
  const char *cwd = nullptr, *out = nullptr, *err = nullptr;
  int pdeathsig = SIGKILL;
  if (!PyArg_ParseTupleAndKeywords(args, kw, "OO|zzzi", const_cast<char**>(kwlist), &py_argv,
                                   &py_env, &cwd, &out, &err, &pdeathsig))
    return nullptr;
  std::vector<std::string> argv_s, env_s;
  if (!to_strings(py_argv, &argv_s, "argv must be a sequence of str")) return nullptr;
  if (!to_strings(py_env, &env_s, "env must be a sequence of 'K=V' str")) return nullptr;
  if (argv_s.empty()) {
    PyErr_SetString(PyExc_ValueError, "argv must not be empty");
    return nullptr;
  }
  std::vector<char*> argv, envp;
  for (auto& s : argv_s) argv.push_back(const_cast<char*>(s.c_str()));
  argv.push_back(nullptr);
  const char* path = nullptr;
  for (auto& s : env_s) {
    envp.push_back(const_cast<char*>(s.c_str()));
    if (s.compare(0, 5, "PATH=") == 0) path = s.c_str() + 5;
  }
  envp.push_back(nullptr);
  int pfd[2];
  if (pipe2(pfd, O_CLOEXEC) != 0) return PyErr_SetFromErrno(PyExc_OSError);
  const pid_t parent = getpid();
  // fork() with the GIL HELD and no Py_BEGIN/END_ALLOW_THREADS around it: the
  // child must never try to re-acquire the GIL (another parent thread may own
  // it at fork time -> the child would deadlock before execve).
  pid_t pid = fork();
  if (pid < 0) {
    close(pfd[0]);
    close(pfd[1]);
    return PyErr_SetFromErrno(PyExc_OSError);
  }
  if (pid == 0) {
    // ---- child: async-signal-safe calls only
    setsid();
    if (pdeathsig > 0) {
      prctl(PR_SET_PDEATHSIG, pdeathsig);
      if (getppid() != parent) _exit(137);  // parent died between fork and prctl
    }
    sigset_t none;
    sigemptyset(&none);
    sigprocmask(SIG_SETMASK, &none, nullptr);
    int devnull = open("/dev/null", O_RDONLY);
    if (devnull >= 0) {
      dup2(devnull, 0);
      if (devnull > 2) close(devnull);
    }
    int fo = -1, fe = -1;
    if (out) fo = open(out, O_WRONLY | O_CREAT | O_APPEND, 0644);
    if (err) fe = (out && strcmp(out, err) == 0) ? fo : open(err, O_WRONLY | O_CREAT | O_APPEND, 0644);
    if (fo >= 0) dup2(fo, 1);
    if (fe >= 0) dup2(fe, 2);
    if (fo > 2) close(fo);
    if (fe > 2 && fe != fo) close(fe);
    if (cwd && *cwd && chdir(cwd) != 0) {
      int e = errno;
      ssize_t w = write(pfd[1], &e, sizeof(e));
      (void)w;
      _exit(126);
    }
    exec_search(argv[0], argv.data(), envp.data(), path);
    int e = errno;
    ssize_t w = write(pfd[1], &e, sizeof(e));
    (void)w;
    _exit(e == ENOENT ? 127 : 126);
  }
  // ---- parent
  close(pfd[1]);
  int child_errno = 0;
  ssize_t n;
  Py_BEGIN_ALLOW_THREADS
  do {
    n = read(pfd[0], &child_errno, sizeof(child_errno));
  } while (n < 0 && errno == EINTR);
  Py_END_ALLOW_THREADS
  close(pfd[0]);
  if (n == static_cast<ssize_t>(sizeof(child_errno))) {
    // exec failed; reap the child and raise with its errno
    int st;
    waitpid(pid, &st, 0);
    errno = child_errno;
    PyObject* msg = PyUnicode_FromFormat("exec %s: %s", argv_s[0].c_str(), strerror(child_errno));
    PyObject* exc = PyObject_CallFunction(PyExc_OSError, "iO", child_errno, msg);
    Py_XDECREF(msg);
    if (exc) {
      PyErr_SetObject(PyExc_OSError, exc);
      Py_DECREF(exc);
    }
    return nullptr;
  }
  return PyLong_FromLong(pid);
}

int exit_code_of(int st) {
  if (WIFEXITED(st)) return WEXITSTATUS(st);
  if (WIFSIGNALED(st)) return 128 + WTERMSIG(st);
  return -1;
}

PyObject* py_reap(PyObject*, PyObject* arg) {
  PyObject* fast = PySequence_Fast(arg, "pids must be a sequence of int");
  if (!fast) return nullptr;
  PyObject* res = PyList_New(0);
  Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
  for (Py_ssize_t i = 0; i < n; ++i) {
    long pid = PyLong_AsLong(PySequence_Fast_GET_ITEM(fast, i));
    if (pid == -1 && PyErr_Occurred()) {
      Py_DECREF(fast);
      Py_DECREF(res);
      return nullptr;
    }
    int st = 0;
    pid_t r = waitpid(static_cast<pid_t>(pid), &st, WNOHANG);
    if (r == static_cast<pid_t>(pid)) {
      PyObject* t = Py_BuildValue("(li)", pid, exit_code_of(st));
      PyList_Append(res, t);
      Py_DECREF(t);
    } else if (r < 0 && errno == ECHILD) {
      PyObject* t = Py_BuildValue("(li)", pid, -1);  // not our child / already reaped
      PyList_Append(res, t);
      Py_DECREF(t);
    }
  }
  Py_DECREF(fast);
  return res;
}

PyObject* py_kill_group(PyObject*, PyObject* args) {
  long pid;
  int sig;
  if (!PyArg_ParseTuple(args, "li", &pid, &sig)) return nullptr;
  if (pid <= 0) {
    PyErr_SetString(PyExc_ValueError, "pid must be > 0");
    return nullptr;
  }
  int r = killpg(static_cast<pid_t>(pid), sig);
  if (r != 0 && errno == ESRCH) r = kill(static_cast<pid_t>(pid), sig);
  return PyLong_FromLong(r == 0 ? 0 : -errno);
}

PyObject* py_alive(PyObject*, PyObject* arg) {
  long pid = PyLong_AsLong(arg);
  if (pid == -1 && PyErr_Occurred()) return nullptr;
  int r = kill(static_cast<pid_t>(pid), 0);
  return PyBool_FromLong(r == 0 || errno == EPERM);
}

// Make this process a child subreaper: orphaned descendants (ranks forked by
// the pre-warmed zygote and double-forked away from it) are re-parented to us,
// so the supervisor can waitpid() them like directly spawned ranks.
PyObject* py_set_child_subreaper(PyObject*, PyObject*) {
  if (prctl(PR_SET_CHILD_SUBREAPER, 1) != 0) return PyErr_SetFromErrno(PyExc_OSError);
  Py_RETURN_NONE;
}

PyMethodDef methods[] = {
    {"set_child_subreaper", py_set_child_subreaper, METH_NOARGS,
     "set_child_subreaper() -> None (PR_SET_CHILD_SUBREAPER on this process)"},
    {"spawn", reinterpret_cast<PyCFunction>(py_spawn), METH_VARARGS | METH_KEYWORDS,
     "spawn(argv, env, cwd=None, out=None, err=None, pdeathsig=SIGKILL) -> pid"},
    {"reap", py_reap, METH_O, "reap(pids) -> [(pid, exit_code)] for exited children (non-blocking)"},
    {"kill_group", py_kill_group, METH_VARARGS, "kill_group(pid, sig) -> 0 or -errno"},
    {"alive", py_alive, METH_O, "alive(pid) -> bool"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

extern "C" PyObject* kdl_native_alloc_module_init(PyObject* m);

static PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_native",
                             "kubedl_amd native runtime primitives (process supervisor, GPU allocator)",
                             -1, methods};

PyMODINIT_FUNC PyInit__native(void) {
  PyObject* m = PyModule_Create(&moddef);
  if (!m) return nullptr;
  if (!kdl_native_alloc_module_init(m)) {
    Py_DECREF(m);
    return nullptr;
  }
  return m;
}
