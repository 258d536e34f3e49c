"""NodeProvider interface. Parity: reference python/ray/autoscaler/node_provider.py (the subset the
autoscaler loop uses: list / tag / create / terminate nodes)."""
from __future__ import annotations

from typing import Any, Dict, List, Optional


class NodeProvider:
    def __init__(self, provider_config: Dict[str, Any], cluster_name: str):
        self.provider_config = provider_config
        self.cluster_name = cluster_name

    def non_terminated_nodes(self, tag_filters: Dict[str, str]) -> List[str]:
        raise NotImplementedError

    def is_running(self, node_id: str) -> bool:
        raise NotImplementedError

    def is_terminated(self, node_id: str) -> bool:
        return not self.is_running(node_id)

    def node_tags(self, node_id: str) -> Dict[str, str]:
        raise NotImplementedError

    def set_node_tags(self, node_id: str, tags: Dict[str, str]) -> None:
        raise NotImplementedError

    def internal_ip(self, node_id: str) -> str:
        return "127.0.0.1"

    def external_ip(self, node_id: str) -> Optional[str]:
        return None

    def create_node(self, node_config: Dict[str, Any], tags: Dict[str, str], count: int) -> Optional[Dict[str, Any]]:
        raise NotImplementedError

    def terminate_node(self, node_id: str) -> None:
        raise NotImplementedError

    def terminate_nodes(self, node_ids: List[str]) -> None:
        for n in node_ids:
            self.terminate_node(n)
