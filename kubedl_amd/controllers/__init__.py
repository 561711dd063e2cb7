"""Per-framework workload controllers (``controllers/``) and their registry
(``controllers/controllers.go`` + ``add_*.go``: kind -> reconciler)."""
from kubedl_amd.controllers.pytorch import PyTorchJobReconciler
from kubedl_amd.controllers.tensorflow import TFJobReconciler
from kubedl_amd.controllers.xdl import XDLJobReconciler
from kubedl_amd.controllers.xgboost import XGBoostJobReconciler

RECONCILERS = {
    "TFJob": TFJobReconciler,
    "PyTorchJob": PyTorchJobReconciler,
    "XGBoostJob": XGBoostJobReconciler,
    "XDLJob": XDLJobReconciler,
}

__all__ = ["RECONCILERS", "TFJobReconciler", "PyTorchJobReconciler", "XGBoostJobReconciler",
           "XDLJobReconciler"]
