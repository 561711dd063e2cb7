# kdl runtime image: ROCm 7 + PyTorch-ROCm base, kernels built for gfx950 at
# image build time (the reference's Dockerfile:1-29 builds a static Go manager).
FROM rocm/pytorch:latest
ENV PYTORCH_ROCM_ARCH=gfx950 \
    HSA_ENABLE_IPC_MODE_LEGACY=0 \
    KDL_HOME=/var/lib/kdl
WORKDIR /opt/kdl
COPY . /opt/kdl
RUN python -m kubedl_amd.ops.build && python -c "import kubedl_amd._C, kubedl_amd._native"
ENV PATH=/opt/kdl/bin:$PATH
EXPOSE 8080 8443
ENTRYPOINT ["kdl", "manager"]
CMD ["--metrics-addr", ":8443", "--gang-scheduler-name", "kdl-gang"]
