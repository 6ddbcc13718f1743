'use strict';
// The JS wrapper's fast paths (js/index.js): launchNetwork encodes the values
// itself and hands the addon typed arrays (networkCreateTyped), and
// getNodesState decodes raw bo_node_state records (getStatesRaw).  Both must
// give exactly what the addon's per-element paths (networkCreate, getStates)
// give: the same errors in the same order (launchNodes.ts:10-13) and the same
// NodeState objects.  No GPU: pre-run states only.
const path = require('path');
const assert = require('assert');
const addon = require(path.join(__dirname, '..', '..', 'ben-or-consensus-algorithm_amd', 'js', 'benor.node'));
const benor = require(path.join(__dirname, '..', '..', 'ben-or-consensus-algorithm_amd', 'js', 'index.js'));

function slow(N, F, init, faulty) {
  try {
    return { states: addon.getStates(addon.networkCreate(N, F, init, faulty)).states };
  } catch (e) {
    return { error: e.message };
  }
}

async function fast(N, F, init, faulty) {
  try {
    await benor.launchNetwork(N, F, init, faulty);
    return { states: await benor.getNodesState(N) };
  } catch (e) {
    return { error: e.message };
  }
}

const cases = [
  [5, 1, [1, 1, 1, 0, 0], [false, false, false, false, true]],
  [5, 1, [1, 0, '?', 1, 0], [true, false, false, false, false]],
  [4, 3, ['?', 1, 0, 1], [true, true, true, false]],
  [3, 0, [0, 1, 2], [false, false, false]],                 // 2 is not a Value
  [3, 0, [-0, 1.0, '1'], [false, false, false]],            // -0 is 0, '1' is not a Value
  [3, 1, [true, 0, 1], [1, true, false]],                   // booleans are not Values; faulty counts `=== true` only
  [3, 1, [1, 0], [true, false, false]],                     // Arrays don't match
  [3, 1, [1, 0, 1], [false, false, false]],                 // faultyList doesnt have F faulties
  [0, 0, [], []],
  [64, 21, Array.from({ length: 64 }, (_, i) => i % 3 === 2 ? '?' : i % 2), Array.from({ length: 64 }, (_, i) => i < 21)],
];

(async () => {
  for (const [N, F, init, faulty] of cases) {
    const a = slow(N, F, init, faulty), b = await fast(N, F, init, faulty);
    assert.deepStrictEqual(b, a, JSON.stringify({ N, F, init, faulty }));
  }
  const r = await benor.getNodesStateAt(64);
  assert.strictEqual(r.events, null);
  assert.strictEqual(r.states.length, 64);
  console.log(`typed paths: ${cases.length} cases agree`);
})().catch((e) => { console.error(e); process.exit(1); });
