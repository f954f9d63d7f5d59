"""MI355X-native ML platform with the capabilities of the Kubeflow control plane
(AnandPolamarasetti/service-account-auth-improvements) plus a gfx950 data plane.

Subpackages:
  ops/          hand-written CDNA4 HIP kernels (K1-K8) + fp32 references
  models/       Llama-3 model family (training + decode)
  parallel/     DP (bucketed RCCL all-reduce / ZeRO-1), TP, PP over xGMI
  runtime/      flat parameter storage, optimizer, trainer, checkpointing, predictor
  controlplane/ Kubeflow-compatible CRDs, controllers, webhooks, KFAM, web backends
  native/       C++ launcher / rendezvous agent
"""
__version__ = "0.1.0"
