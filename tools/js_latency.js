'use strict';
// The reference's own calls from JavaScript (the drop-in's N-API path):
// launchNetwork + startConsensus (default: resolves at launch) + waitConsensus
// + getNodesState, and the reference tests' pattern of polling getNodesState
// until reachedFinality (benorconsensus.test.ts:153-160, utils.ts:14-24).
// One JSON line per (N, F, form): median and p90 wall time in ms.
//
//   node tools/js_latency.js [reps]
const path = require('path');
const benor = require(path.join(__dirname, '..', 'ben-or-consensus-algorithm_amd', 'js', 'index.js'));

const now = () => Number(process.hrtime.bigint()) / 1e6;

async function main() {
  const reps = Number(process.argv[2] || 60);
  for (const [N, F] of [[5, 1], [10, 4], [10, 5], [100, 33], [1024, 341]]) {
    const init = Array.from({ length: N }, (_, i) => (i * 7 + 3) % 2);
    const faulty = Array.from({ length: N }, (_, i) => i < F);
    const n = N >= 1024 ? Math.max(5, Math.floor(reps / 5)) : reps;
    for (const form of ['wait', 'poll', 'sync']) {
      if (form === 'poll' && F * 2 >= N) continue;   // no decision: the poll would run to k_max
      const times = [];
      let last = null;
      for (let r = 0; r < n + 3; r++) {
        const t0 = now();
        await benor.launchNetwork(N, F, init, faulty);
        await benor.startConsensus(N, { seed: r, sync: form === 'sync' });
        if (form === 'poll') {
          last = await benor.getNodesState(N);
          while (!benor.reachedFinality(last)) last = await benor.getNodesState(N);
          await benor.waitConsensus(N);
        } else {
          await benor.waitConsensus(N);
          last = await benor.getNodesState(N);
        }
        if (r >= 3) times.push(now() - t0);
      }
      times.sort((a, b) => a - b);
      const decided = last.filter((s) => s.decided).length;
      console.log(JSON.stringify({ N, F, form, reps: n, median_ms: times[times.length >> 1],
                                   p90_ms: times[Math.floor(times.length * 0.9)], last_decided_nodes: decided }));
    }
  }
}

main().catch((e) => { console.error(e); process.exit(1); });
