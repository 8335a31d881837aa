// nbd_ops.cpp — operator schemas of the nbdistributed_amd HIP kernels (torch.ops.nbd.*).
// The GPU implementations are registered next to their kernels (bucket.hip, summary.hip) under
// the CUDA dispatch key (HIP on ROCm).  CPU tensors are served by the PyTorch reference
// implementations in nbdistributed_amd/ops (same semantics; used by the CPU test-suite).
#include <torch/library.h>

TORCH_LIBRARY(nbd, m) {
  m.def("bucket_flatten(Tensor[] tensors, Tensor(a!) bucket, int[] offsets, float scale, bool accumulate=False) -> ()");
  m.def("bucket_unflatten(Tensor bucket, Tensor(a!)[] tensors, int[] offsets, float scale, bool accumulate) -> ()");
  m.def("local_prereduce(Tensor[] inputs, Tensor(a!) out, float scale) -> ()");
  m.def("tensor_summary(Tensor x) -> Tensor");
  m.def("attn_fwd(Tensor q, Tensor k, Tensor v, bool causal, float scale, Tensor? rope_cos=None, "
        "Tensor? rope_sin=None) -> (Tensor, Tensor)");
  m.def("attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor out, Tensor lse, bool causal, float scale, "
        "Tensor(a!) dq, Tensor(b!) dk, Tensor(c!) dv, Tensor? rope_cos=None, Tensor? rope_sin=None, "
        "Tensor? delta=None) -> ()");
  m.def("decode_attn(Tensor qkv, Tensor(a!) k_cache, Tensor(b!) v_cache, Tensor pos, int n_head, float scale, "
        "int kv_len_max, Tensor? rope_cos, Tensor? rope_sin, Tensor(c!) partials) -> Tensor");
  m.def("greedy_advance(Tensor logits, Tensor(a!) tok, Tensor(b!) pos, Tensor(c!) out, Tensor(d!)? done, int eos) -> ()");
  m.def("linear_small(Tensor x, Tensor w, Tensor? bias, Tensor? norm_w, Tensor? norm_b, float eps, int norm, "
        "int act, Tensor? residual) -> Tensor");
  m.def("attn_merge_(Tensor(a!) o_acc, Tensor(b!) lse_acc, Tensor o_b, Tensor lse_b, Tensor(c!)? out=None) -> ()");
  m.def("ln_fwd(Tensor x, Tensor? delta, Tensor weight, Tensor bias, float eps) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("ln_bwd(Tensor x, Tensor dy, Tensor? dres, Tensor weight, Tensor mean, Tensor rstd) -> (Tensor, Tensor, Tensor)");
  m.def("colsum(Tensor x, ScalarType dtype) -> Tensor");
  m.def("rms_fwd(Tensor x, Tensor? delta, Tensor weight, float eps) -> (Tensor, Tensor, Tensor)");
  m.def("rms_bwd(Tensor x, Tensor dy, Tensor? dres, Tensor weight, Tensor rstd) -> (Tensor, Tensor)");
  m.def("embedding_bwd(Tensor dy, Tensor idx, int V, Tensor(a!)? grad_out=None, bool accumulate=False) -> Tensor");
  m.def("embedding_tokpos(Tensor idx, Tensor wte, Tensor pos, Tensor wpe, int vocab=-1, Tensor(a!)? err=None) -> Tensor");
  m.def("embedding_pos_bwd(Tensor dy, Tensor pos, int P, Tensor(a!)? out=None, bool accumulate=False) -> Tensor");
  m.def("rope_(Tensor(a!) x, Tensor cos, Tensor sin, int n_rot, int head_dim, bool inverse) -> ()");
  m.def("seqcls_prep(Tensor ids, Tensor? mask, int pad_id, bool has_pad, Tensor(a!) bad) -> (Tensor, Tensor)");
  m.def("swiglu_fwd(Tensor gu) -> Tensor");
  m.def("swiglu_bwd(Tensor gu, Tensor dact) -> Tensor");
  m.def("xent_fwd(Tensor logits, Tensor target, int ignore_index) -> (Tensor, Tensor)");
  m.def("xent_bwd(Tensor logits, Tensor target, Tensor lse, Tensor scale, int ignore_index, Tensor(a!) dlogits) -> ()");
  m.def("xent_fused(Tensor(a!) logits, Tensor target, int ignore_index, Tensor scale) -> (Tensor, Tensor)");
  m.def("xent_mean_scale(Tensor target, int ignore_index) -> Tensor");
  m.def("xent_loss_total(Tensor rows, Tensor scale) -> Tensor");
  m.def("scale_pair_(Tensor(a!) a, Tensor b, Tensor g) -> Tensor");
  m.def("gemm(Tensor a, Tensor b, Tensor(a!) c, bool a_km, bool b_kn, Tensor? bias, int epi, Tensor? aux_in, "
        "Tensor(b!)? aux_out, int splits, int tile, int accum=0) -> ()");
  m.def("gemm_pair(Tensor a1, Tensor b1, Tensor(a!) c1, int epi1, Tensor? aux_in1, Tensor a2, Tensor b2, "
        "Tensor(b!) c2, int epi2, Tensor(c!)? aux_out2, int splits2, int accum2=0, Tensor(d!)? delta1=None, "
        "int delta_T=0) -> ()");
  // autograd nodes of the fused Linear / MLP paths (autograd.hip); plan = ops/gemm.py native_plan
  m.def("linear_ag(Tensor x, Tensor w, Tensor? b, int[] plan) -> Tensor");
  m.def("mlp_gelu_ag(Tensor x, Tensor w1, Tensor? b1, Tensor w2, Tensor? b2, int[] plan) -> Tensor");
  m.def("mlp_swiglu_ag(Tensor x, Tensor w_gu, Tensor w_down, int[] plan) -> Tensor");
  m.def("rms_norm_ag(Tensor x, Tensor w, float eps) -> Tensor");
  m.def("add_rms_norm_ag(Tensor x, Tensor delta, Tensor w, float eps) -> (Tensor, Tensor)");
  m.def("embed_rms_norm_ag(Tensor ids, Tensor table, Tensor w, float eps, Tensor(a!)? err=None) -> (Tensor, Tensor)");
  m.def("tokpos_layer_norm_ag(Tensor idx, Tensor wte, Tensor pos, Tensor wpe, Tensor w, Tensor b, int vocab, float eps, "
        "Tensor(a!)? err=None) -> (Tensor, Tensor)");
  m.def("layer_norm_ag(Tensor x, Tensor w, Tensor b, float eps) -> Tensor");
  m.def("add_layer_norm_ag(Tensor x, Tensor delta, Tensor w, Tensor b, float eps) -> (Tensor, Tensor)");
  m.def("attn_qkv_ag(Tensor qkv, int n_head, int n_kv, bool causal, float scale, Tensor? cos, Tensor? sin) -> Tensor");
  m.def("llama_block_ag(Tensor x, Tensor h, Tensor w_qkv, Tensor? b_qkv, Tensor w_o, Tensor? b_o, Tensor w_post, "
        "Tensor w_gu, Tensor w_down, Tensor w_next, int[] plan_qkv, int[] plan_o, int[] plan_mlp, int n_head, int n_kv, "
        "float scale, float eps, Tensor? cos, Tensor? sin, int graphs=-1, int owner=0) -> (Tensor, Tensor)");
  m.def("cast_group_ag(Tensor[] ps, int dtype) -> Tensor[]");
  m.def("adamw_flat_multi(Tensor[] grads, Tensor(a!)[] params, Tensor(b!)[] masters, Tensor(c!)[] exp_avgs, "
        "Tensor(d!)[] exp_avg_sqs, float lr, float beta1, float beta2, float eps, float weight_decay, int step, "
        "float grad_scale, Tensor? grad_scale_t=None, Tensor? step_t=None, Tensor? lr_t=None) -> ()");

  m.def("adamw_tensors(Tensor(a!)[] params, Tensor[] grads, Tensor(b!)[] exp_avgs, Tensor(c!)[] exp_avg_sqs, "
        "Tensor[] steps, float lr, float beta1, float beta2, float eps, float weight_decay) -> ()");
  m.def("adamw_flat(Tensor grad, Tensor(a!) param, Tensor(b!) master, Tensor(c!) exp_avg, Tensor(d!) exp_avg_sq, "
        "float lr, float beta1, float beta2, float eps, float weight_decay, int step, float grad_scale, Tensor? grad_scale_t=None, Tensor? step_t=None, Tensor? lr_t=None) -> ()");
}
