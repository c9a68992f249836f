{{- define "nexus.name" -}}
{{- default .Chart.Name .Values.nameOverride | trunc 63 | trimSuffix "-" -}}
{{- end -}}

{{- define "nexus.fullname" -}}
{{- if .Values.fullnameOverride -}}
{{- .Values.fullnameOverride | trunc 63 | trimSuffix "-" -}}
{{- else -}}
{{- printf "%s-%s" .Release.Name (include "nexus.name" .) | trunc 63 | trimSuffix "-" -}}
{{- end -}}
{{- end -}}

{{- define "nexus.labels" -}}
app.kubernetes.io/name: {{ include "nexus.name" . }}
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/version: {{ .Chart.AppVersion | quote }}
app.kubernetes.io/managed-by: {{ .Release.Service }}
helm.sh/chart: {{ printf "%s-%s" .Chart.Name .Chart.Version }}
{{- with .Values.additionalLabels }}
{{ toYaml . }}
{{- end }}
{{- end -}}

{{- define "nexus.selectorLabels" -}}
app.kubernetes.io/name: {{ include "nexus.name" . }}
app.kubernetes.io/instance: {{ .Release.Name }}
{{- end -}}

{{- define "nexus.serviceAccountName" -}}
{{- if .Values.serviceAccount.create -}}
{{- default (include "nexus.fullname" .) .Values.serviceAccount.name -}}
{{- else -}}
{{- default "default" .Values.serviceAccount.name -}}
{{- end -}}
{{- end -}}

{{- define "nexus.image" -}}
{{- printf "%s:%s" .Values.image.repository (default (printf "v%s" .Chart.AppVersion) .Values.image.tag) -}}
{{- end }}

{{/* node agent image: ROCm base (amd-smi), linux/amd64 (deploy/Dockerfile) */}}
{{- define "nexus.agentImage" -}}
{{- printf "%s:%s" .Values.agent.image.repository (default (printf "v%s" .Chart.AppVersion) .Values.agent.image.tag) -}}
{{- end -}}

{{- /* reference: rbac.clusterRole.supervisor.nameOverride (/root/reference/.helm/templates/_helpers.tpl:77-83) */ -}}
{{- define "nexus.roleName" -}}
{{- $override := .Values.rbac.nameOverride -}}
{{- if .Values.rbac.clusterRole -}}
{{- if .Values.rbac.clusterRole.supervisor -}}
{{- if .Values.rbac.clusterRole.supervisor.nameOverride -}}
{{- $override = .Values.rbac.clusterRole.supervisor.nameOverride -}}
{{- end -}}
{{- end -}}
{{- end -}}
{{- if $override -}}
{{- $override -}}
{{- else -}}
{{- printf "%s-api-access" (include "nexus.fullname" .) -}}
{{- end -}}
{{- end -}}
