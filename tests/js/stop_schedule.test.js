'use strict';
// Mid-run GET /stop through the JavaScript mirror (tests/test_stop_schedule.py
// writes the cases and the oracle's expected per-node states):
//   launchNetwork(N, F, init, faulty) -> startConsensus(N, {seed, kMax, stopAfter})
//   -> getNodesState(N) must equal the expected states.
// Usage: node stop_schedule.test.js cases.json
const fs = require('fs');
const path = require('path');
const assert = require('assert');
const b = require(path.join(__dirname, '..', '..', 'ben-or-consensus-algorithm_amd', 'js', 'index.js'));

async function main() {
  const cases = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
  for (const c of cases) {
    const servers = await b.launchNetwork(c.N, c.F, c.init, c.faulty);
    await b.startConsensus(c.N, { seed: BigInt(c.seed), kMax: c.k_max, stopAfter: c.stopAfter });
    const states = await b.getNodesState(c.N);
    assert.deepStrictEqual(states, c.expect, `N=${c.N} F=${c.F} stops=${JSON.stringify(c.stopAfter)}`);
    for (const node of Object.keys(c.stopAfter)) {
      const st = await b.getNodeStatus(Number(node));
      assert.strictEqual(st.status, 500);                // node.ts:33-39 after the stop
    }
    await Promise.all(servers.map((s) => s.close()));
  }
  console.log(`${cases.length} cases ok`);
}

main().catch((e) => { console.error(e); process.exit(1); });
