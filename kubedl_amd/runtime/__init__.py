"""Local MI355X node runtime: scheduler (GPU binding), kubelet (rank-process
supervisor), service resolver and the image registry."""
