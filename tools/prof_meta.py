"""The bench configuration a tools/profile.sh run measured, read from the run's own bench.py JSON
line (prof_TAG/kt.log), so that tools/pmc_summary.py and tools/trace_summary.py file a run's numbers
under the config it ran (a config-5 run once overwrote the config-3 entry)."""
import json
import os


def bench_meta(prof_dir):
    """(config, samples_per_step) of the bench line in prof_dir/kt.log, or None if absent."""
    p = os.path.join(prof_dir, 'kt.log')
    if not os.path.exists(p):
        return None
    for ln in reversed(open(p, errors='replace').read().splitlines()):
        ln = ln.strip()
        if ln.startswith('{'):
            try:
                rec = json.loads(ln)
            except ValueError:
                continue
            cfg = rec.get('config', {})
            if 'config' in cfg and 'samples_per_step_per_gpu' in cfg:
                return int(cfg['config']), int(cfg['samples_per_step_per_gpu'])
    return None


def resolve_config(prof_dir, config=None):
    """The run's config only (trace summaries): from its bench line, else the explicit value."""
    meta = bench_meta(prof_dir)
    if meta is None:
        if config is None:
            raise SystemExit('%s has no bench line (kt.log): pass --config' % prof_dir)
        return config
    if config is not None and config != meta[0]:
        raise SystemExit('%s measured config %d, not %d' % (prof_dir, meta[0], config))
    return meta[0]


def resolve(prof_dir, config=None, samples=None):
    """The run's (config, samples): from its bench line; explicit values must agree with it, and
    are required when the run has none."""
    meta = bench_meta(prof_dir)
    if meta is None:
        if config is None or samples is None:
            raise SystemExit('%s has no bench line (kt.log): pass --config and --samples-log2' % prof_dir)
        return config, samples
    if config is not None and config != meta[0]:
        raise SystemExit('%s measured config %d, not %d' % (prof_dir, meta[0], config))
    if samples is not None and samples != meta[1]:
        raise SystemExit('%s measured %d samples per step, not %d' % (prof_dir, meta[1], samples))
    return meta
