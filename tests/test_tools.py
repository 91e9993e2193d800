"""CPU tests of the measurement tools whose output is committed under profiles/ (no GPU)."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trace(path, rows):
    with open(path, 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['Kind', 'Kernel_Name', 'Start_Timestamp', 'End_Timestamp'])
        for name, s, e in rows:
            w.writerow(['KERNEL_DISPATCH', name, s, e])


def test_step_timeline_splits_steps_and_counts_idle(tmp_path):
    """tools/step_timeline.py: steps split at the per-step kernel, idle = the part of a step no kernel covers."""
    rows = []
    t = 0
    for step in range(5):
        rows.append(('pjaccard_partial', t, t + 10_000))           # 10 us
        rows.append(('igemm_halo16_x3<1,4>', t + 10_000, t + 500_000))  # back to back
        rows.append(('bn_stats_finalize', t + 503_000, t + 509_000))    # 3 us gap before it
        t += 510_000                                                  # 1 us to the next step
    p = tmp_path / 'run_kernel_trace.csv'
    _trace(p, rows)
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'step_timeline.py'), str(p),
                          '--per-step-kernel', 'pjaccard_partial', '--skip', '1', '--list'],
                         capture_output=True, text=True, check=True).stdout
    assert 'steps analysed: 3 (skipped 1)' in out
    assert 'wall per step       0.510 ms' in out
    assert 'kernel-covered      0.506 ms' in out
    assert 'idle between        0.004 ms' in out
    assert 'launches / step  3' in out
    assert 'bn_stats_finalize' in out


def test_step_stats_counts_steady_state_steps_only(tmp_path):
    """tools/step_stats.py on a kernel trace: one-time launches before the steady state (AdamW's first-step state
    fills, parameter copies) are not spread over the steps; each kept step holds exactly its own launches."""
    rows = []
    t = 0
    for i in range(40):  # one-time setup work before and inside the first (warmup) step
        rows.append(('at::native::vectorized_elementwise_kernel<4, at::native::FillFunctor<float>>', t, t + 1_000))
        t += 1_000
    for step in range(6):
        rows.append(('void scd::igemm_halo16_x3<1, 4>(scd::IgemmArgs)', t, t + 400_000))
        rows.append(('void scd::pjaccard_partial(float)', t + 400_000, t + 410_000))
        rows.append(('void scd::bn_stats_finalize(float)', t + 410_000, t + 416_000))
        if step == 0:
            rows.append(('__amd_rocclr_copyBuffer', t + 416_000, t + 417_000))
        t += 420_000
    p = tmp_path / 'run_kernel_trace.csv'
    _trace(p, rows)
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'step_stats.py'), str(p),
                          '--per-step-kernel', 'pjaccard_partial', '--skip', '2'],
                         capture_output=True, text=True, check=True).stdout
    assert 'steady state: the 3 steps after the first 2 (kernel trace)' in out
    assert 'conv kernels      0.400 ms/step' in out
    assert 'FillFunctor' not in out and 'copyBuffer' not in out
    assert '    1.00' in out  # one launch of each per step
