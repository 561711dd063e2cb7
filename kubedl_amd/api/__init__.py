"""Public job API: kubeflow/KubeDL CRD schemas, defaulting and codec."""
from kubedl_amd.api import common, kinds, codec  # noqa: F401
from kubedl_amd.api.kinds import (ALL_KINDS, BY_KIND, PYTORCHJOB, TFJOB, XDLJOB,  # noqa: F401
                                  XGBOOSTJOB, KindInfo, lookup, replica_specs, run_policy,
                                  set_defaults, validate)
