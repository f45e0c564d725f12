"""Stand-in for graph-theory 2022.4.3 (`graph.Graph`, poetry.lock pin), used ONLY to import the
reference in this container.  PARITY ASSUMPTION (documented in DESIGN.md, "parity unpinned"):
edges are stored as a nested dict {n1: {n2: value}} in insertion order, so `edges()` is grouped by
source node in the order sources were first used; `shortest_path` is heap Dijkstra with a FIFO
insertion counter as tie-break, neighbours visited in `edges(from_node=...)` order."""
from collections import deque
from heapq import heappop, heappush


class Graph:
    def __init__(self):
        self._nodes = {}
        self._edges = {}

    def add_node(self, node_id, obj=None):
        self._nodes[node_id] = obj

    def add_edge(self, node1, node2, value=1, bidirectional=False):
        if node1 not in self._nodes:
            self.add_node(node1)
        if node2 not in self._nodes:
            self.add_node(node2)
        self._edges.setdefault(node1, {})[node2] = value
        if bidirectional:
            self.add_edge(node2, node1, value, False)

    def del_edge(self, node1, node2):
        d = self._edges[node1]
        del d[node2]

    def edges(self, from_node=None):
        if from_node is not None:
            return [(from_node, n2, v) for n2, v in self._edges.get(from_node, {}).items()]
        return [(n1, n2, v) for n1, d in self._edges.items() for n2, v in d.items()]

    def nodes(self, from_node=None):
        if from_node is not None:
            return list(self._edges.get(from_node, {}).keys())
        return list(self._nodes)

    def __contains__(self, item):
        return item in self._nodes

    def breadth_first_search(self, start, end):
        parent = {start: None}
        q = deque([start])
        while q:
            n = q.popleft()
            if n == end:
                path = []
                while n is not None:
                    path.append(n)
                    n = parent[n]
                return path[::-1]
            for n2 in self._edges.get(n, {}):
                if n2 not in parent:
                    parent[n2] = n
                    q.append(n2)
        return []

    def is_connected(self, start, end):
        return bool(self.breadth_first_search(start, end))

    def shortest_path(self, start, end):
        q = [(0, 0, start, ())]
        minimums = {start: 0}
        visited = set()
        i = 1
        while q:
            cost, _, v1, path = heappop(q)
            if v1 in visited:
                continue
            visited.add(v1)
            path = (v1, path)
            if v1 == end:
                out = []
                while path:
                    out.append(path[0])
                    path = path[1]
                return cost, out[::-1]
            for _, v2, dist in self.edges(from_node=v1):
                if v2 in visited:
                    continue
                nxt = cost + dist
                prev = minimums.get(v2)
                if prev is None or nxt < prev:
                    minimums[v2] = nxt
                    heappush(q, (nxt, i, v2, path))
                    i += 1
        return float("inf"), []
