'use strict';
// GET /stop during a live run through the JavaScript mirror
// (tests/test_live_stop.py writes the cases and checks the results against
// the oracle for the recorded delivery counts):
//   launchNetwork -> startConsensus(N, {seed, kMax: 16, live: true}) -> stopNode(i)
//   -> waitConsensus(N) -> getNodesState(N) -> liveStopEvents(N)
// Usage: node live_stop.test.js cases.json out.json
const fs = require('fs');
const path = require('path');
const assert = require('assert');
const b = require(path.join(__dirname, '..', '..', 'ben-or-consensus-algorithm_amd', 'js', 'index.js'));

async function main() {
  const cases = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
  const results = [];
  for (const c of cases) {
    const servers = await b.launchNetwork(c.N, c.F, c.init, c.faulty);
    await b.startConsensus(c.N, { seed: BigInt(c.seed), kMax: 16, live: true });
    for (const i of c.stops) {
      await b.stopNode(i);
      const st = await b.getNodeStatus(i);
      assert.strictEqual(st.status, 500);              // node.ts:33-39, answered mid-run
    }
    await b.waitConsensus(c.N);
    const states = await b.getNodesState(c.N);
    const events = await b.liveStopEvents(c.N);
    results.push({ states, events });
    await Promise.all(servers.map((s) => s.close()));
  }
  fs.writeFileSync(process.argv[3], JSON.stringify(results));
  console.log(`${cases.length} cases ran`);
}

main().catch((e) => { console.error(e); process.exit(1); });
