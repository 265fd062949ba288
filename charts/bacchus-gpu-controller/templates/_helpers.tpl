{{/* Chart name, truncated to the 63-char DNS label limit. */}}
{{- define "bgc.name" -}}
{{- default .Chart.Name .Values.controller.nameOverride | trunc 63 | trimSuffix "-" }}
{{- end }}

{{/* Release-qualified name; the release name alone when it already contains the chart name. */}}
{{- define "bgc.fullname" -}}
{{- if .Values.controller.fullnameOverride }}
{{- .Values.controller.fullnameOverride | trunc 63 | trimSuffix "-" }}
{{- else }}
{{- $name := include "bgc.name" . }}
{{- if contains $name .Release.Name }}
{{- .Release.Name | trunc 63 | trimSuffix "-" }}
{{- else }}
{{- printf "%s-%s" .Release.Name $name | trunc 63 | trimSuffix "-" }}
{{- end }}
{{- end }}
{{- end }}

{{- define "bgc.chart" -}}
{{- printf "%s-%s" .Chart.Name .Chart.Version | replace "+" "_" | trunc 63 | trimSuffix "-" }}
{{- end }}

{{/* Selector labels. `component` keeps each Deployment/Service selecting only its own
     pods (the reference shared one selector, so its webhook Service also routed to the
     plain-HTTP controller/synchronizer pods). Call with (dict "root" $ "component" "x"). */}}
{{- define "bgc.selectorLabels" -}}
app.kubernetes.io/name: {{ include "bgc.name" .root }}
app.kubernetes.io/instance: {{ .root.Release.Name }}
app.kubernetes.io/component: {{ .component }}
{{- end }}

{{- define "bgc.labels" -}}
helm.sh/chart: {{ include "bgc.chart" .root }}
{{ include "bgc.selectorLabels" . }}
app.kubernetes.io/version: {{ .root.Chart.AppVersion | quote }}
app.kubernetes.io/managed-by: {{ .root.Release.Service }}
{{- end }}

{{- define "bgc.authorizedGroups" -}}
{{- join "," .Values.admission.configs.authorized_group_names }}
{{- end }}
