"""Shared helpers (the reference's ``pkg/util`` tree, SURVEY.md §2.7 "util misc",
"k8sutil", "tenancy / quota / signals").

- ``log``:      job / replica / pod / key loggers with structured fields
                (``pkg/util/logger.go:26-80``)
- ``k8sutil``:  pod filtering, replica totals, owner and replica-type lookup
                (``pkg/util/k8sutil/k8sutil.go:95-160``)
- ``quota``:    container resource sum / max (``pkg/util/quota/resources.go:8-35``)
- ``tenancy``:  the ``kubedl.io/tenancy`` annotation (``pkg/util/tenancy/tenancy.go:25-43``)
- ``misc``:     ``pformat``, ``rand_string``, namespace env (``pkg/util/util.go``)
- ``signals``:  SIGINT/SIGTERM -> stop event, second signal exits
                (``pkg/util/signals/signal.go:27-43``)
"""
