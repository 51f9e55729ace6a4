"""Where does configs[4]'s bf16 G-gradient error enter?  

One trainer G-step at B = 32 (p = 0, fixed labels, the models of
tests/test_gpu_configs.py::test_bf16_train_step_b32), gradients of every G parameter compared with
the all-fp32 step (global cosine over the parameters with a non-zero true gradient, and the
median per-weight cosine), for variants that put bf16 GEMM operands in one place at a time:

  - the forward pass only / the backward pass only;
  - the forward of one module group only (forward pre/post hooks switch the engine precision;
    backward in fp32);
  - bf16x6 (fp32-class operands, a different rounding): the step's own noise floor;
  - the fp32 step with the generated pose perturbed by relative noise eps (a forward hook): how
    strongly the loss gradient reacts to a forward perturbation of that size, independent of
    where it comes from.

    python tools/bf16_grad_probe.py [--out gpurun_out/bf16_grad_probe.jsonl]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'audio-to-motion-generation_amd'), os.path.join(REPO, 'tests')]

import numpy as np  # noqa: E402
import torch  # noqa: E402

DEV = torch.device('cuda:0')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', default=None)
    a = ap.parse_args()
    import a2m
    from a2m import autograd as AG
    from a2m.model_layers import SelfAttention
    from a2m.training import GANTrainer, compute_temporal_smoothness_loss_and_jerk
    from oracle import synth
    from test_gpu_configs import _models
    from test_gpu_train import _bn_cancelled

    gen = torch.Generator().manual_seed(21)
    audio = (torch.randn(32, 64, 128, generator=gen) * 2.0 - 3.0).to(DEV)
    pose = torch.from_numpy(synth.pose_targets(32, 64, seed=22)).to(DEV)

    orig_cna = AG.conv_norm_act
    layer_prec = {}      # id(ConvNormRelu) -> precision, for layers AG calls without module hooks

    def cna(m, x, out=None):
        p = layer_prec.get(id(m))
        if p is None:
            return orig_cna(m, x, out=out)
        prev = a2m.set_gemm_precision(p)
        try:
            return orig_cna(m, x, out=out)
        finally:
            a2m.set_gemm_precision(prev)
    AG.conv_norm_act = cna

    def step(fwd='fp32', bwd='fp32', groups=None, eps=0.0, enc_layers=None):
        """groups: (module selector, precision) forward overrides; enc_layers: {encoder conv
        index: precision} forward overrides of single AudioEncoder layers."""
        g, d = _models(DEV)
        layer_prec.clear()
        for i, p in (enc_layers or {}).items():
            layer_prec[id(g.audio_encoder.conv[i])] = p
        tr = GANTrainer(g, d, lr=0.0, fixed_labels=(0.93, 0.07))
        valid, _ = tr._labels(0, 32, DEV)
        for p_ in d.parameters():
            p_.requires_grad_(False)
        hooks, stack = [], []
        for sel, prec in (groups or []):
            for m in sel(g, d):
                hooks.append(m.register_forward_pre_hook(
                    lambda mod, inp, prec=prec: stack.append(a2m.set_gemm_precision(prec))))
                hooks.append(m.register_forward_hook(lambda mod, inp, out: (a2m.set_gemm_precision(stack.pop()), None)[1]))
        if eps:
            gn = torch.Generator(device=DEV).manual_seed(5)

            def perturb(mod, inp, out):
                pose_, internal = out
                return pose_ + eps * pose_.detach().abs().max() * torch.randn(pose_.shape, generator=gn, device=DEV), internal
            hooks.append(g.register_forward_hook(perturb))
        with a2m.gemm_precision(fwd):
            fake_pose, internal = g(audio, real_pose=pose)
            fake_d, _ = d(AG.pos_to_motion(fake_pose))
            terms = compute_temporal_smoothness_loss_and_jerk(fake_pose, pose)
            loss = terms[0] + tr.lambda_gan * AG.mse_loss(fake_d, valid) + 0.1 * terms[1] + 0.05 * terms[2]
            for t in internal:
                loss = loss + t
        for h in hooks:
            h.remove()
        with a2m.gemm_precision(bwd):
            loss.backward()
        torch.cuda.synchronize()
        grads = {n: p_.grad.detach().double().flatten().clone() for n, p_ in g.named_parameters() if p_.grad is not None}
        dims = {n: p_.dim() for n, p_ in g.named_parameters()}
        return grads, dims, fake_pose.detach(), loss.item()

    ref, dims, ref_pose, ref_loss = step()

    def agree(b):
        names = [n for n in ref if not _bn_cancelled(n) and ref[n].norm() > 0]
        x, y = torch.cat([ref[n] for n in names]), torch.cat([b[n] for n in names])
        glob = (torch.dot(x, y) / (x.norm() * y.norm())).item()
        per = {n: (torch.dot(ref[n], b[n]) / (ref[n].norm() * b[n].norm())).item() for n in names}
        med = float(np.median([v for n, v in per.items() if dims[n] >= 2]))
        worst = sorted(per.items(), key=lambda kv: kv[1])[:5]
        return glob, med, worst

    attn = lambda g, d: [m for m in g.modules() if isinstance(m, SelfAttention)]  # noqa: E731
    variants = [
        ('fp32 again (determinism)', dict()),
        ('bf16x6 fwd+bwd (noise floor)', dict(fwd='bf16x6', bwd='bf16x6')),
        ('bf16 fwd+bwd (configs[4])', dict(fwd='bf16', bwd='bf16')),
        ('bf16 fwd, fp32 bwd', dict(fwd='bf16')),
        ('fp32 fwd, bf16 bwd', dict(bwd='bf16')),
        ('bf16 fwd: audio_encoder only', dict(groups=[(lambda g, d: [g.audio_encoder], 'bf16')])),
        ('bf16 fwd: unet only', dict(groups=[(lambda g, d: [g.unet], 'bf16')])),
        ('bf16 fwd: body decoder only', dict(groups=[(lambda g, d: [g.body_decoder_pre, g.body_decoder_post], 'bf16')])),
        ('bf16 fwd: hand decoder only', dict(groups=[(lambda g, d: [g.hand_decoder_pre, g.hand_decoder_post], 'bf16')])),
        ('bf16 fwd: discriminator only', dict(groups=[(lambda g, d: [d], 'bf16')])),
        ('bf16 fwd: SelfAttention modules only', dict(groups=[(attn, 'bf16')])),
        ('bf16 fwd+bwd, SelfAttention forward fp32', dict(fwd='bf16', bwd='bf16', groups=[(attn, 'fp32')])),
        ('bf16 fwd+bwd, discriminator forward fp32', dict(fwd='bf16', bwd='bf16', groups=[(lambda g, d: [d], 'fp32')])),
        ('bf16 fwd+bwd, encoder conv0 forward fp32', dict(fwd='bf16', bwd='bf16', enc_layers={0: 'fp32'})),
        ('bf16 fwd+bwd, encoder conv0-1 forward fp32', dict(fwd='bf16', bwd='bf16', enc_layers={0: 'fp32', 1: 'fp32'})),
        ('bf16 fwd+bwd, audio_encoder forward fp32', dict(fwd='bf16', bwd='bf16', groups=[(lambda g, d: [g.audio_encoder], 'fp32')])),
        ('bf16 fwd+bwd, audio_encoder + SelfAttention forward fp32', dict(fwd='bf16', bwd='bf16', groups=[(lambda g, d: [g.audio_encoder], 'fp32'), (attn, 'fp32')])),
        ('bf16 fwd+bwd, audio_encoder + unet forward fp32', dict(fwd='bf16', bwd='bf16', groups=[(lambda g, d: [g.audio_encoder, g.unet], 'fp32')])),
    ] + [(f'fp32, pose perturbed by {e:g} x max|pose|', dict(eps=e)) for e in (1e-6, 1e-5, 1e-4, 1e-3, 1e-2)]
    out = open(a.out, 'w') if a.out else None
    # layer trace: every ConvNormRelu / attention / decoder module's forward output in bf16 vs
    # fp32 (same input weights, train mode), plus, for conv + train-mode BatchNorm layers, the
    # worst channel's |mean| / std of the pre-BN conv output in fp32 -- a BN over a channel whose
    # spread is tiny against its mean turns the operands' 2^-9 rounding into |mean|/std x 2^-9
    from a2m.model_layers import ConvNormRelu, ChannelAttention, ResBlock, ConvTranspose1D
    kinds = (ConvNormRelu, SelfAttention, ChannelAttention, ResBlock, ConvTranspose1D)

    def trace(prec):
        g, d = _models(DEV)
        rec, hooks = [], []
        enc_ids = {id(m): i for i, m in enumerate(g.audio_encoder.conv)}

        def cna_rec(m, x, out=None):
            y = orig_cna(m, x, out=out)
            if id(m) in enc_ids:
                entry = {'name': f'audio_encoder.conv.{enc_ids[id(m)]}', 'out': y.detach().clone()}
                with torch.no_grad():
                    pre = m.conv(x.detach()).double()
                mu, sd = pre.mean([0, 2, 3]), pre.std([0, 2, 3])
                entry['mean_over_std'] = float((mu.abs() / sd.clamp_min(1e-30)).max())
                rec.append(entry)
            return y
        AG.conv_norm_act = cna_rec
        for n, m in list(g.named_modules()) + [('D.' + n, m) for n, m in d.named_modules()]:
            if isinstance(m, kinds):
                def hk(mod, inp, o, n=n):
                    entry = {'name': n, 'out': (o[0] if isinstance(o, (tuple, list)) else o).detach().clone()}
                    if isinstance(mod, ConvNormRelu) and getattr(mod, 'norm', None) is not None and \
                            isinstance(mod.conv, (torch.nn.Conv1d, torch.nn.Conv2d)):
                        with torch.no_grad():
                            pre = mod.conv(inp[0].detach()).double()
                        dims = [0] + list(range(2, pre.dim()))
                        mu, sd = pre.mean(dims), pre.std(dims)
                        entry['mean_over_std'] = float((mu.abs() / sd.clamp_min(1e-30)).max())
                    rec.append(entry)
                hooks.append(m.register_forward_hook(hk))
        try:
            with a2m.gemm_precision(prec), torch.no_grad():
                fp, _ = g(audio, real_pose=pose)
                d(AG.pos_to_motion(fp))
        finally:
            AG.conv_norm_act = cna
        for h in hooks:
            h.remove()
        return rec
    t32, t16 = trace('fp32'), trace('bf16')
    for r32, r16 in zip(t32, t16):
        e = ((r16['out'] - r32['out']).abs().max() / r32['out'].abs().max().clamp_min(1e-30)).item()
        rec = {'layer': r32['name'], 'bf16_rel_err': float(f'{e:.3e}')}
        if 'mean_over_std' in r32:
            rec['pre_bn_max_mean_over_std'] = round(r32['mean_over_std'], 2)
        print(json.dumps(rec), flush=True)
        if out:
            out.write(json.dumps(rec) + '\n')
    for name, kw in variants:
        gr, _, fp, loss = step(**kw)
        glob, med, worst = agree(gr)
        perr = ((fp - ref_pose).abs().max() / ref_pose.abs().max()).item()
        rec = {'variant': name, 'g_cos_global': round(glob, 5), 'g_cos_weight_median': round(med, 5),
               'pose_rel_err': float(f'{perr:.3e}'), 'g_loss': loss, 'g_loss_fp32': ref_loss,
               'worst5': [(n, round(v, 4)) for n, v in worst]}
        print(json.dumps(rec), flush=True)
        if out:
            out.write(json.dumps(rec) + '\n')
    if out:
        out.close()


if __name__ == '__main__':
    main()
